// Helpers shared by the fold kernels (kernels.hip, mfe_cells.hip): cell
// indexing of the DP tables, pair types, the LDS-only barrier, the packed
// 16-bit min-plus encoding and the per-cell table block layout.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace adx {
namespace {

constexpr int WAVE = 64;

// index of the first cell of diagonal dd (cells with j - i = dd >= 4)
__device__ __forceinline__ int off(int dd, int N) { return ((dd - 4) * (2 * N - 3 - dd)) >> 1; }

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Workgroup barrier ordering LDS only (the fold's waves share nothing else
// inside its diagonal loop): outstanding global loads are not drained, so a
// prefetch issued before the barrier completes in the shadow of the next
// iteration instead of stalling the barrier.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Workgroup OR of v through the LDS word *w, which must hold 0 and have been
// written before a barrier every thread has passed since.  Replaces
// __syncthreads_or, whose library implementation adds 256 B of static LDS:
// with none, the dynamic LDS starts at address 0 and every carve address is a
// literal the compiler rematerialises instead of keeping it in an SGPR.
__device__ __forceinline__ bool block_or(int *w, bool v) {
    if (__ballot(v) != 0 && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(w, 1);
    __syncthreads();
    return *w != 0;
}

// The walker a fold workgroup takes at launch position wb (order: a step's
// launch order, kernels.hip order_kernel; null: blockIdx order), or -1 when
// mask (1 = fold) leaves it nothing to fold.
__device__ __forceinline__ int walker_at(const int *order, const int *mask, int wb) {
    const int w = order ? order[wb] : wb;
    if (mask && mask[w] != 1) return -1;
    return w;
}

// A fold workgroup's per-walker words -- its mask, slot index, slot validity and
// the proposal's changed range -- loaded in one round trip after the walker's index
// (the chain order -> mask -> slot -> change waited on three); valid is false and
// c0 < 0 without incremental state.  K: KArgs (dev_types.hpp)
struct WalkerRef {
    int w, cur, c0, c1;
    bool on, valid;
};
template <class K>
__device__ __forceinline__ WalkerRef walker_ref(const K &ka, const int *mask, int wb) {
    WalkerRef r;
    r.w = ka.order ? ka.order[wb] : wb;
    const int w = r.w;
    const int mk = mask ? mask[w] : 1;
    r.cur = ka.tab ? int(ka.cur_slot[w]) : 0;
    r.valid = ka.tab ? ka.tab_valid[w] != 0 : false;
    r.c0 = ka.chg ? ka.chg[2 * w] : -1;
    r.c1 = ka.chg ? ka.chg[2 * w + 1] : -1;
    r.on = mk == 1;
    return r;
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
constexpr int MFE16_FLOOR = -12000;
// Exactness of the packed 16-bit MFE encoding (kernels.hip MinPlus16): a half
// >= 0x4000 is "impossible".  A true finite value can only reach that band as
// a sum of at most two stored values plus loop constants (each < 40.96
// kcal/mol, i.e. < 0x1000), so while every stored finite value is below
// MFE16_CEIL = 0x1800 (61.44 kcal/mol) no finite value is ever mistaken for an
// impossible one; and an impossible operand plus one stored value >= FLOOR
// stays >= 0x7FFF - 12000 > 0x4000, so no impossible value passes for finite.
// A fold with a stored half outside [FLOOR, CEIL) -- other than the impossible
// band [0x4000, 0x7FFF] -- is re-folded by the FP32 kernel (round 6: the
// ceiling; before, a forced fold above 163.84 kcal/mol read as impossible).
constexpr int MFE16_CEIL = 0x1800;
__device__ __forceinline__ bool mfe16_inexact(s16x2 q) {
    auto out = [](int h) { return h < MFE16_FLOOR || (h >= MFE16_CEIL && h < 0x4000); };
    return out(q.x) || out(q.y);
}

// Index of the special hairpin whose key is `key` in spk[0, MAX_SPECIAL_HP) (LDS,
// 16-byte aligned, padded with 0xFFFFFFFF, which hp_key never returns), or -1; the
// last match, as a scan would find.  Every key comes in wave-uniform 16-byte loads
// issued before any compare: the compare -> value-load chain per key it replaces
// serialised ~16 LDS round trips per 8 keys, ~10k cycles per cell-pass item on the
// special-hairpin diagonals (stamps, profiles/r06s_mfe_pair_stamps_setup.txt)
__device__ __forceinline__ int special_hp(const uint32_t *spk, uint32_t key) {
    static_assert(MAX_SPECIAL_HP % 16 == 0, "whole 16-key chunks");
    int hit = -1;
#pragma unroll
    for (int q0 = 0; q0 < MAX_SPECIAL_HP; q0 += 16) {
        uint4 k[4];
#pragma unroll
        for (int t = 0; t < 4; t++) k[t] = reinterpret_cast<const uint4 *>(spk + q0)[t];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            hit = k[t].x == key ? q0 + 4 * t : hit;
            hit = k[t].y == key ? q0 + 4 * t + 1 : hit;
            hit = k[t].z == key ? q0 + 4 * t + 2 : hit;
            hit = k[t].w == key ? q0 + 4 * t + 3 : hit;
        }
    }
    return hit;
}

// Pair type / reversed type / terminal-AU flag without a memory lookup:
// PAIR[a][b] for codes a, b in 0..4 (ViennaRNA types 1..6) packed 3 bits per
// entry of index 5a+b-9 (the canonical pairs sit at 9..23).
constexpr unsigned long long pack_pairs() {
    unsigned long long k = 0;
    k |= 5ull << (3 * (9 - 9));    // A-U
    k |= 1ull << (3 * (13 - 9));   // C-G
    k |= 2ull << (3 * (17 - 9));   // G-C
    k |= 3ull << (3 * (19 - 9));   // G-U
    k |= 6ull << (3 * (21 - 9));   // U-A
    k |= 4ull << (3 * (23 - 9));   // U-G
    return k;
}
__device__ __forceinline__ int ptype(int a, int b) {
    const int idx = 5 * a + b - 9;
    return (idx >= 0 && idx <= 14) ? int((pack_pairs() >> (3 * idx)) & 7ull) : 0;
}
__device__ __forceinline__ int rtype(int t) { return t ? (((t - 1) ^ 1) + 1) : 0; }

// Cell indexing (1-based i < j, span j - i >= 4):
//   qbm, cc  diagonal-major  off(j-i) + i - 1   (cells of one anti-diagonal contiguous)
//   qm       row-major       rowb(i) + j - i - 4 (qm[i][*] contiguous)
//   qm1      column-major    colb(j) + i - 1     (qm1[*][j] contiguous)
// so every inner loop of the recurrence walks contiguous LDS at a per-lane base.
__device__ __forceinline__ int rowb(int i, int N) { return (i - 1) * (N - 3) - (((i - 1) * i) >> 1); }
__device__ __forceinline__ int colb(int j) { return ((j - 5) * (j - 4)) >> 1; }

// LDS per-cell table block (L.dt), copied from DevTables / DevScaled
constexpr int DT_MMH = 0;      // [type][x][y] hairpin mismatch
constexpr int DT_MMI = 200;    // [type][x][y] interior mismatch
constexpr int DT_MLS = 400;    // [type][x][y] multiloop stem
constexpr int DT_EXT = 600;    // [type][6][6] exterior stem
constexpr int DT_TAU = 888;    // [type] terminal AU
constexpr int DT_HP = 896;     // [u] hairpin length factor

}  // namespace
}  // namespace adx
