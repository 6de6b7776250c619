// ipc_k_fp32.hip — the one-sided kernels for Fp32 (ipc_kernel_body.h; one translation unit per dtype group so the
// instantiations compile in parallel).
#include "ipc_kernel_body.h"

namespace hccl_amd {

HCCL_AMD_IPC_DTYPE(Fp32, EFp<float>)

}  // namespace hccl_amd
