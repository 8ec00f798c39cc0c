// wave_ops.h -- cross-lane reductions for one 64-lane wave on gfx950, through
// DPP (row_shr / row_bcast VALU modifiers) instead of LDS permutes: a 6-step
// ds_bpermute reduction of a double costs ~800 cycles on MI355X
// (tools/microbench.hip), the DPP form a small fraction of that.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace tdstar {

// A load through an address-space-1 (global) pointer: `global_load`, counted in
// vmcnt only.  The same load through a generic pointer is a `flat_load`, counted
// in lgkmcnt too -- and every LDS wait and block barrier (which waits on
// lgkmcnt) would then wait for it.  p must point to device global memory.
template <class T>
__device__ __forceinline__ T gload(const T *p) {
    return *(const __attribute__((address_space(1))) T *)(p);
}

template <class T>
__device__ __forceinline__ void gstore(T *p, T v) {
    *(__attribute__((address_space(1))) T *)(p) = v;
}

// LDS writes of this wave visible to its own later reads (no block barrier)
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- cross-lane reductions on 64-bit keys through DPP (VALU, no LDS) ----
// A non-negative double orders like its bit pattern, so distances reduce as
// unsigned 64-bit keys.  update_dpp returns `old` in lanes whose source is out
// of the row or masked off, so `old` is the identity of the reduction.
template <int CTRL, int RM>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v, unsigned long long idn) {
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)idn, (int)(unsigned)v, CTRL, RM, 0xf, false);
    const int hi =
        __builtin_amdgcn_update_dpp((int)(unsigned)(idn >> 32), (int)(unsigned)(v >> 32), CTRL, RM, 0xf, false);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
// min over the 64 lanes of the wave, returned to every lane
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    constexpr unsigned long long I = ~0ull;
    v = umin64(v, dpp_u64<0x111, 0xf>(v, I));  // row_shr:1
    v = umin64(v, dpp_u64<0x112, 0xf>(v, I));  // row_shr:2
    v = umin64(v, dpp_u64<0x114, 0xf>(v, I));  // row_shr:4
    v = umin64(v, dpp_u64<0x118, 0xf>(v, I));  // row_shr:8  -> lane 15 of a row: row min
    v = umin64(v, dpp_u64<0x142, 0xa>(v, I));  // row_bcast:15 into rows 1, 3
    v = umin64(v, dpp_u64<0x143, 0xc>(v, I));  // row_bcast:31 into rows 2, 3 -> lane 63: min
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}
// min over the 64 lanes of 32-bit unsigned values, returned to every lane (one DPP min per step)
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
    constexpr int I = -1;  // ~0u
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(I, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}
// wave_min_u64 as two 32-bit passes: the high words' minimum, then (only if several lanes hold it)
// the low words' among those lanes -- the same 64-bit minimum, in a third of the dependent VALU steps
__device__ __forceinline__ unsigned long long wave_min_u64_2p(unsigned long long v) {
    const unsigned hi = (unsigned)(v >> 32), lo = (unsigned)v;
    const unsigned mh = wave_min_u32(hi);
    const unsigned long long at = __ballot(hi == mh);
    unsigned ml;
    if (__popcll(at) == 1) ml = (unsigned)__builtin_amdgcn_readlane((int)lo, __builtin_ctzll(at));  // (wave-uniform)
    else ml = wave_min_u32(hi == mh ? lo : ~0u);
    return ((unsigned long long)mh << 32) | ml;
}
// max over each row of 16 lanes, valid in the row's last lane (lane % 16 == 15)
__device__ __forceinline__ unsigned long long row_max_u64(unsigned long long v) {
    v = umax64(v, dpp_u64<0x111, 0xf>(v, 0ull));
    v = umax64(v, dpp_u64<0x112, 0xf>(v, 0ull));
    v = umax64(v, dpp_u64<0x114, 0xf>(v, 0ull));
    v = umax64(v, dpp_u64<0x118, 0xf>(v, 0ull));
    return v;
}
// xor over the 64 lanes, to every lane
__device__ __forceinline__ unsigned long long wave_xor_u64(unsigned long long v) {
    v ^= dpp_u64<0x111, 0xf>(v, 0ull);
    v ^= dpp_u64<0x112, 0xf>(v, 0ull);
    v ^= dpp_u64<0x114, 0xf>(v, 0ull);
    v ^= dpp_u64<0x118, 0xf>(v, 0ull);
    v ^= dpp_u64<0x142, 0xa>(v, 0ull);  // row_bcast:15
    v ^= dpp_u64<0x143, 0xc>(v, 0ull);  // row_bcast:31 -> lane 63: the whole wave
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// inclusive prefix sum over the 64 lanes (lane l: v_0 + ... + v_l, in a tree
// association: exact when every value and partial sum is an integer < 2^53).
// The row shifts zero-fill (bound_ctrl); the row broadcasts leave the
// unselected rows at `old` = 0.
__device__ __forceinline__ double wave_scan_f64(double v) {
    auto shr = [](double a, auto ctrl) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(a);
        const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, decltype(ctrl)::value, 0xf, 0xf, true);
        const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), decltype(ctrl)::value, 0xf, 0xf, true);
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    };
    auto bits = [](double a) { return (unsigned long long)__double_as_longlong(a); };
    v = v + shr(v, std::integral_constant<int, 0x111>{});  // row_shr 1, 2, 4, 8: scan inside rows of 16
    v = v + shr(v, std::integral_constant<int, 0x112>{});
    v = v + shr(v, std::integral_constant<int, 0x114>{});
    v = v + shr(v, std::integral_constant<int, 0x118>{});
    v = v + __longlong_as_double((long long)dpp_u64<0x142, 0xa>(bits(v), 0ull));  // row_bcast:15 -> rows 1, 3
    v = v + __longlong_as_double((long long)dpp_u64<0x143, 0xc>(bits(v), 0ull));  // row_bcast:31 -> rows 2, 3
    return v;
}

// sum over the 64 lanes (any association: for bounds, not for results), to every lane
__device__ __forceinline__ double wave_sum_f64(double v) {
    auto add = [](double a, unsigned long long b) { return a + __longlong_as_double((long long)b); };
    auto bits = [](double a) { return (unsigned long long)__double_as_longlong(a); };
    v = add(v, dpp_u64<0x111, 0xf>(bits(v), 0ull));  // row_shr: inclusive scan inside rows
    v = add(v, dpp_u64<0x112, 0xf>(bits(v), 0ull));
    v = add(v, dpp_u64<0x114, 0xf>(bits(v), 0ull));
    v = add(v, dpp_u64<0x118, 0xf>(bits(v), 0ull));
    v = add(v, dpp_u64<0x142, 0xa>(bits(v), 0ull));  // row_bcast:15
    v = add(v, dpp_u64<0x143, 0xc>(bits(v), 0ull));  // row_bcast:31 -> lane 63: the total
    return readlane_f64(v, 63);
}

}  // namespace tdstar
