// ipc_k_int.hip — the one-sided kernels for Int8, Int16, Int32 (ipc_kernel_body.h; one translation unit per dtype group so the
// instantiations compile in parallel).
#include "ipc_kernel_body.h"

namespace hccl_amd {

HCCL_AMD_IPC_DTYPE(Int8, EInt<int8_t, uint32_t>)
HCCL_AMD_IPC_DTYPE(Int16, EInt<int16_t, uint32_t>)
HCCL_AMD_IPC_DTYPE(Int32, EInt<int32_t, uint32_t>)

}  // namespace hccl_amd
