// Helpers shared by the lanes = cells MFE kernels (mfe_cells.hip: one
// anti-diagonal per barrier; mfe_pair.hip: two): the packed 16-bit min-plus
// encoding (apo | holo halves), wave reductions, the LDS address of an object
// and the per-lane state the generated interior-loop blocks (mfe_blocks.inc,
// mfe_pair_blocks.inc; tools/gen_mfe_blocks.py) read.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {
namespace {

using u32 = uint32_t;
constexpr u32 INF16 = 0x7FFF7FFFu;
constexpr u32 MARK16 = 0x7FFE7FFEu;   // non-pairable cell (setup value; a finished cell never takes it)

__device__ __forceinline__ s16x2 sv(u32 x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ u32 su(s16x2 x) { return __builtin_bit_cast(u32, x); }
__device__ __forceinline__ u32 pmin(u32 a, u32 b) { return su(__builtin_elementwise_min(sv(a), sv(b))); }
__device__ __forceinline__ u32 padd(u32 a, u32 b) { return su(__builtin_elementwise_add_sat(sv(a), sv(b))); }
__device__ __forceinline__ u32 pfin(u32 u) {   // halves in [0x4000, 0x7FFF] -> 0x7FFF
    const u32 imp = (u & ~(u >> 1)) & 0x40004000u;
    return u | ((imp >> 14) * 0x7FFFu);
}

template <int CTRL, int ROWS>
__device__ __forceinline__ u32 dpp_min(u32 v) {
    const int moved = __builtin_amdgcn_update_dpp(int(INF16), int(v), CTRL, ROWS, 0xf, false);
    return pmin(v, u32(moved));
}
__device__ __forceinline__ u32 wave_min(u32 v) {   // full-wave min, result uniform
    v = dpp_min<0xb1, 0xf>(v);    // quad_perm [1,0,3,2]
    v = dpp_min<0x4e, 0xf>(v);    // quad_perm [2,3,0,1]
    v = dpp_min<0x114, 0xf>(v);   // row_shr:4
    v = dpp_min<0x118, 0xf>(v);   // row_shr:8
    v = dpp_min<0x142, 0xa>(v);   // row_bcast:15
    v = dpp_min<0x143, 0xc>(v);   // row_bcast:31
    return u32(__builtin_amdgcn_readlane(int(v), 63));
}

// min across lane halves / 16-lane rows (lanes l, l^32 / l, l^16 end equal; no LDS)
__device__ __forceinline__ u32 fold_halves(u32 v) {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return pmin(u32(p[0]), u32(p[1]));
}
__device__ __forceinline__ u32 fold_rows16(u32 v) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return pmin(u32(p[0]), u32(p[1]));
}

// LDS byte address of an LDS object (the inline-asm read batches address LDS directly)
typedef __attribute__((address_space(3))) char lds_char;
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T *p) {
    return uint32_t(uintptr_t((lds_char *)(p)));   // generic -> LDS address space
}

// A pointer to LDS byte address a: kernels without static LDS (no __shared__
// variables, no library code that declares any -- fold_common.hpp block_or)
// get their dynamic block at address 0, so a carve of literal addresses needs
// no SGPR per region (the launcher checks the static size is 0)
template <class T>
__device__ __forceinline__ T *lds_at(size_t a) {
    return (T *)((__attribute__((address_space(3))) char *)(uint32_t(a)));
}

template <class LT>
__device__ __forceinline__ bool allowed(const LT &L, int i, int j) {   // kernels.hip allowed()
    const int fi = L.flg[i], fj = L.flg[j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[i], pj = L.ptn[j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[i] == L.enc[j];
}

// The per-size energy records (DevScaled::ku16) through the constant address
// space: uniform loads from it are scalar (s_load, lgkmcnt).  Through a generic
// pointer they were flat loads, which count on vmcnt too, so the first record
// use of a block waited for the block's 1x1..2x2 table prefetches from L2.
#ifndef ADX_KFLAT
typedef __attribute__((address_space(4))) const uint32_t kc_u32;
#else   // A/B knob: the records through a generic pointer (flat loads), as before round 6
typedef const uint32_t kc_u32;
#endif
__device__ __forceinline__ const kc_u32 *kconst(const uint4 *p) { return (const kc_u32 *)(uintptr_t)p; }
__device__ __forceinline__ uint4 kload(const kc_u32 *p, int k) {   // record k (4 words)
    return make_uint4(p[4 * k], p[4 * k + 1], p[4 * k + 2], p[4 * k + 3]);
}

// ---------------------------------------------------------------- interior-loop shapes
struct BUni {                 // wave-uniform
    uint32_t aq, ac, act;     // LDS byte addresses of qbm, cc, ct (inline-asm batches)
    const u32 *qbm;           // LDS
    const uint8_t *cc;        // LDS
    const u32 *ct;            // LDS (per-lane indexed factors)
    const uint4 *kg;          // per loop size u: {il[u] + nin[k] (k = 0..5), bulge[u], 1 x (u-1)}
                              // (DevScaled::ku16, uniform: scalar loads)
    const u32 *gct;           // HBM ctab (uniform entries, runtime path only)
    const u32 *il, *nin;      // HBM generic interior energy parts (runtime path only)
    u32 fs1;                  // bulge of size 1
    int d, N, umax;
    bool mk;                  // some lane's unpaired runs cut loop sizes <= umax: mask shapes
    __device__ __forceinline__ int offu(int u) const { return off(d - 2 - u, N); }
};
struct BCell {                // per lane: the closing pair (i, i+d)
    int i, ty8, A, B;
    uint32_t rs;              // 4 * lane slice (sliced blocks: first generic shape offset)
    uint32_t ee;              // 4 lanes per cell: LDS byte address of the slice's column of CL::e4
    bool r1, r2;              // lane slice bits
    int hb;                   // pair kernel (mfe_pair.hip): 1 on the lanes of the step's second diagonal
    int ea, eb, ctb;          // sliced blocks: the slice's edge shapes n1 = ea + eb * u, their factor table
    u32 m23f;                 // 2x3: interior[5] + ninio + outer mismatch23
    u32 t11, t12, t21, t22;   // prefetched 1x1 / 1x2 / 2x1 / 2x2 table energies
};
struct Acc {
    u32 s, g0, g1, b, n;      // specials; generic (+ outer mismatchI, even / odd u1); bulges (+ TermAU); 1xn (+ mismatch1n)
    u32 e;                    // 4 lanes per cell: the slice's edge shapes (+ TermAU on slices 0, 1, mismatch1n on 2, 3)
};

#define MFE_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)

}  // namespace
}  // namespace adx
