// reduce_elem.h — device-side element rules shared by the reduce kernels (reduce_kernels.hip) and the one-sided
// IPC AllReduce kernel (ipc_kernel_body.h). See reduce_kernels.hip for the reference semantics they restate.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "internal.h"

namespace hccl_amd {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------ element rules

template <typename T, typename W>
struct EInt {
    using S = T;
    template <int OP>
    static __device__ __forceinline__ T ap(T s, T d)
    {
        if constexpr (OP == R_SUM) {
            return static_cast<T>(static_cast<W>(static_cast<W>(s) + static_cast<W>(d)));
        } else if constexpr (OP == R_PROD) {
            return static_cast<T>(static_cast<W>(static_cast<W>(s) * static_cast<W>(d)));
        } else if constexpr (OP == R_MAX) {
            return (s < d) ? d : s;
        } else {
            return (d < s) ? d : s;
        }
    }
};

template <typename T>
struct EFp {
    using S = T;
    template <int OP>
    static __device__ __forceinline__ T ap(T s, T d)
    {
        if constexpr (OP == R_SUM) {
            return s + d;
        } else if constexpr (OP == R_PROD) {
            return s * d;
        } else if constexpr (OP == R_MAX) {
            return (s < d) ? d : s;
        } else {
            return (d < s) ? d : s;
        }
    }
};

// fp16: a native half add/mul is correctly rounded, which equals the reference's fp32-compute + RNE narrowing
// (11-bit significands: 24 >= 2*11+2, so the double rounding is innocuous; products are exact in fp32).
// MAX/MIN compare (exact) and return the selected operand's bits, as the reference's round trip does.
struct EF16 {
    using S = uint16_t;
    template <int OP>
    static __device__ __forceinline__ uint16_t ap(uint16_t s, uint16_t d)
    {
        _Float16 hs = __builtin_bit_cast(_Float16, s);
        _Float16 hd = __builtin_bit_cast(_Float16, d);
        if constexpr (OP == R_SUM) {
            return __builtin_bit_cast(uint16_t, static_cast<_Float16>(hs + hd));
        } else if constexpr (OP == R_PROD) {
            return __builtin_bit_cast(uint16_t, static_cast<_Float16>(hs * hd));
        } else if constexpr (OP == R_MAX) {
            return (hs < hd) ? d : s;
        } else {
            return (hd < hs) ? d : s;
        }
    }
};

// bf16: fp32 compute, round to nearest even (no in-tree reference arithmetic: parity unpinned, SURVEY §8a').
struct EBF16 {
    using S = uint16_t;
    static __device__ __forceinline__ float widen(uint16_t b) { return __builtin_bit_cast(float, uint32_t(b) << 16); }
    // v_cvt_pk_bf16_f32: round to nearest even in hardware, a NaN stays a NaN (MI355X_MICROARCH.md, correctness
    // boundaries). The integer rounding sequence it replaces made bf16 SUM VALU-bound (5.3 vs 6.3 TB/s).
    static __device__ __forceinline__ uint16_t narrow(float f)
    {
        return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
    }
    template <int OP>
    static __device__ __forceinline__ uint16_t ap(uint16_t s, uint16_t d)
    {
        float fs = widen(s);
        float fd = widen(d);
        if constexpr (OP == R_SUM) {
            return narrow(fs + fd);
        } else if constexpr (OP == R_PROD) {
            return narrow(fs * fd);
        } else if constexpr (OP == R_MAX) {
            return (fs < fd) ? d : s;
        } else {
            return (fd < fs) ? d : s;
        }
    }
};

template <class E, int OP>
__device__ __forceinline__ u32x4 combine(u32x4 s, u32x4 d)
{
    using S = typename E::S;
    if constexpr (std::is_same<E, EInt<int8_t, uint32_t>>::value && OP == R_SUM) {
        // int8 SUM, four lanes per dword without unpacking: add the low 7 bits of every byte (no carry can cross a
        // byte), then put back each byte's top bit as the XOR of the operands' top bits and that carry. Two's
        // complement wrap per byte, the same bits as the per-element rule.
        u32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t a = s[i], b = d[i];
            r[i] = ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
        }
        return r;
    }
    constexpr int N = 16 / sizeof(S);
    S a[N];
    S b[N];
    __builtin_memcpy(a, &s, 16);
    __builtin_memcpy(b, &d, 16);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        a[i] = E::template ap<OP>(a[i], b[i]);
    }
    u32x4 r;
    __builtin_memcpy(&r, a, 16);
    return r;
}

// NT is a bit set: bit 0 = non-temporal loads, bit 1 = non-temporal stores.
template <int NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr ((NT & 1) != 0) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

template <int NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr ((NT & 2) != 0) {
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

}  // namespace hccl_amd
