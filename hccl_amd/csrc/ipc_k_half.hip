// ipc_k_half.hip — the one-sided kernels for Fp16, Bf16 (ipc_kernel_body.h; one translation unit per dtype group so the
// instantiations compile in parallel).
#include "ipc_kernel_body.h"

namespace hccl_amd {

HCCL_AMD_IPC_DTYPE(Fp16, EF16)
HCCL_AMD_IPC_DTYPE(Bf16, EBF16)

}  // namespace hccl_amd
