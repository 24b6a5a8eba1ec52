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

// The walker a fold workgroup takes at launch position wb (order: a step's
// launch order, kernels.hip order_kernel; null: blockIdx order), or -1 when
// mask (1 = fold) leaves it nothing to fold.
__device__ __forceinline__ int walker_at(const int *order, const int *mask, int wb) {
    const int w = order ? order[wb] : wb;
    if (mask && mask[w] != 1) return -1;
    return w;
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
constexpr int MFE16_FLOOR = -12000;

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
