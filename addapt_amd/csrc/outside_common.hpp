// Shared by the lanes = cells outside kernels (outside_cells.hip for N <= 112,
// outside_ring.hip beyond): the LDS view, the interior-loop shape machinery of
// the B waves (one window read per shape at a per-lane base + immediate
// offset) and the B sweep, templated on the lane-sets a diagonal may need.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "dev_types.hpp"
#include "fold_common.hpp"

#ifndef OSTAMP
#define OSTAMP(k) do { } while (0)
#endif

namespace adx {
namespace {

constexpr int OX_NW = 16;             // waves per workgroup
constexpr int OX_NT = OX_NW * WAVE;
constexpr int OX_NB = 10;             // interior-loop blocks (waves 0..9)
constexpr int OX_NM = OX_NW - OX_NB;  // multiloop-sum waves (10..15)
constexpr int OX_WIN = 32;            // qbb window: spans d+2 .. d+32 are read at step d
constexpr int OX_PAD = 32;            // zero cells in front of each window row (outer a >= i-31)
constexpr int OX_MAXP = 64;           // requested pairs of one fold kept in LDS
constexpr int OX_FF = 5;              // finalize record fields (see frec_write)
constexpr int OX_RF = 8;              // cell setup record fields (see rec_write)

struct OxL {
    float *yr, *yc, *q1r, *qmc, *qw, *part, *mlp, *rec, *fr, *sf, *rq, *rr, *r1, *q5, *q5b, *pm, *ct, *dt;
    int *pl;
    uint8_t *ow, *S, *mat, *cl;
    int *rcnt;
    double *pd;
    int RL, NP;
};

__device__ __forceinline__ int wslot(int D) { return D & (OX_WIN - 1); }

// diagonal D of the diagonal-major cell index k: off(D) <= k < off(D + 1)
__device__ __forceinline__ int inv_off(int k, int N) {
    const float b = float(2 * N - 7);
    int D = 4 + int((b - sqrtf(fmaxf(b * b - 8.f * float(k), 0.f))) * 0.5f);
    D = D < 4 ? 4 : D;
    while (D < N - 1 && off(D + 1, N) <= k) D++;
    while (D > 4 && off(D, N) > k) D--;
    return D;
}
// column j of the column-major cell index k: colb(j) <= k < colb(j + 1)
__device__ __forceinline__ int inv_colb(int k) {
    int j = 5 + int((sqrtf(8.f * float(k) + 1.f) - 1.f) * 0.5f);
    while (colb(j + 1) <= k) j++;
    while (colb(j) > k) j--;
    return j;
}

// interior-loop shape kinds (dev_types.hpp TermKind; -1 = generic)
__host__ __device__ constexpr int okind(int n1, int n2) {
    return (n1 == 0 && n2 == 0) ? TK_STK
         : (n1 + n2 == 1) ? TK_B1
         : (n1 == 0 || n2 == 0) ? TK_BUL
         : (n1 == 1 && n2 == 1) ? TK_I11
         : (n1 == 1 && n2 == 2) ? TK_I12
         : (n1 == 2 && n2 == 1) ? TK_I21
         : (n1 == 2 && n2 == 2) ? TK_I22
         : ((n1 == 2 && n2 == 3) || (n1 == 3 && n2 == 2)) ? TK_M23
         : (n1 == 1 || n2 == 1) ? TK_1N
         : -1;
}

struct OxCell {                 // per lane: the inner pair (i, j) of every shape
    int i;
    float mmin, tau_in, mo_in, m23_in;
    float t11, t12, t21, t22;   // 1x1 / 1x2 / 2x1 / 2x2 table factors (HBM, issued at the block start)
};

// One shape (N1, U - N1) of the lane's cell; qw / ow: this lane's window row of
// the outer span d + 2 + U at outer a = i - 1 - U (n1 = U), so shape N1 reads
// offset U - N1; fv: the shapes' constant factors (OxL::sf row U, in registers).
// Compile-time shape: the kind and every table offset fold.
template <int U, int N1>
__device__ __forceinline__ void oshape1(const OxL &L, const OxCell &c, const float *fv, const float *qw,
                                        const uint8_t *ow, int ty2, float &g, float &sp) {
    constexpr int k = okind(N1, U - N1);
    const float v = qw[U - N1];
    if constexpr (k < 0) {
        g = fmaf(v, fv[N1], g);
    } else {
        const float *ct = L.ct;
        const int oc = ow[U - N1];
        float f;
        if constexpr (k == TK_STK || k == TK_B1) {
            f = ct[CT_INVMM + oc] * ct[CT_STK + ((oc * 41) >> 10) * 8 + ty2] * fv[N1];
        } else if constexpr (k == TK_BUL) {
            f = ct[CT_BUL + oc] * (c.tau_in * fv[N1]);
        } else if constexpr (k == TK_1N) {
            f = ct[CT_ONEN + oc] * (c.mo_in * fv[N1]);
        } else if constexpr (k == TK_M23) {
            f = ct[CT_INVMM + oc] * ct[CT_M23O + oc] * (c.m23_in * fv[N1]);
        } else {
            const float tv = k == TK_I11 ? c.t11 : k == TK_I12 ? c.t12 : k == TK_I21 ? c.t21 : c.t22;
            f = ct[CT_INVMM + oc] * (tv * fv[N1]);
        }
        sp = fmaf(v, f, sp);
    }
}
template <int U, int... N1s>
__device__ __forceinline__ void oshape_seq(std::integer_sequence<int, N1s...>, const OxL &L, const OxCell &c,
                                           const float *fv, const float *qw, const uint8_t *ow, int ty2, float &g,
                                           float &sp) {
    (oshape1<U, N1s>(L, c, fv, qw, ow, ty2, g, sp), ...);
}
// the shapes of loop size U (skipped past the step's umax: uniform)
template <int U>
struct OxSize {
    float fv[U < 0 ? 1 : U + 1];
    __device__ __forceinline__ void load(const OxL &L) {
        if constexpr (U >= 0)
#pragma unroll
            for (int n1 = 0; n1 <= U; n1++) fv[n1] = L.sf[U * 32 + n1];
    }
    __device__ __forceinline__ void run(const OxL &L, const OxCell &c, int d, int umax, int ty2, float &g,
                                        float &sp) const {
        if constexpr (U >= 0) {
            if (U <= umax) {
                const int o = wslot(d + 2 + U) * L.RL + OX_PAD + c.i - 2 - U;
                oshape_seq<U>(std::make_integer_sequence<int, U + 1>{}, L, c, fv, L.qw + o, L.ow + o, ty2, g, sp);
            }
        }
    }
};

// Loop size U >= 6 over the four lanes of an inner cell (phase r = lane & 3),
// as pf_cells.hip PxSizeQ: lane r takes one special shape -- the bulges (0,U)
// (U,0) and 1 x n loops (1,U-1) (U-1,1), a window read, an outer-code read and
// a factor gather -- and the generic shapes n1 = 2 + r + 4m <= U - 2 (one
// window read at a per-lane base + immediate offset, its factor in a VGPR; 0
// past the size).  The four lanes' sums are added in a fixed order.
template <int U>
struct OxSizeQ {
    static constexpr int NR = U >= 6 ? (U - 3 + 3) / 4 : 1;
    float gf[NR];
    float fsp;
    int n1sp;
    __device__ __forceinline__ void load(const OxL &L, int r) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const int n1 = 2 + 4 * m + r;
            gf[m] = n1 <= U - 2 ? L.sf[U * 32 + n1] : 0.f;
        }
        n1sp = r == 0 ? 0 : r == 1 ? U : r == 2 ? 1 : U - 1;
        fsp = L.sf[U * 32 + n1sp];
    }
    __device__ __forceinline__ void run(const OxL &L, const OxCell &c, int d, int umax, int ctb, float outer,
                                        float &g, float &sp) const {
        if (U <= umax) {
            const int o = wslot(d + 2 + U) * L.RL + OX_PAD + c.i - 2 - U;   // shape n1 at o + U - n1
            {
                const float v = L.qw[o + U - n1sp];
                const int oc = L.ow[o + U - n1sp];
                sp = fmaf(v, L.ct[ctb + oc] * (outer * fsp), sp);
            }
            const float *q = L.qw + o + U - 2 - (threadIdx.x & 3);
#pragma unroll
            for (int m = 0; m < NR; m++) g = fmaf(q[-4 * m], gf[m], g);
        }
    }
};
#ifndef ADX_SMALL_R0
#define ADX_SMALL_R0 1   // sizes <= 5 on phase 0 only (the other phases' copies are discarded)
#endif
template <int U>
struct OxBlk {   // the size's state in a B wave (sizes <= 5 whole in every lane)
    using T = typename std::conditional<(U <= 5), OxSize<U>, OxSizeQ<U>>::type;
};
template <int U>
__device__ __forceinline__ void ox_load(typename OxBlk<U>::T &z, const OxL &L, int r) {
    if constexpr (U <= 5) z.load(L);
    else z.load(L, r);
}
template <int U>
__device__ __forceinline__ void ox_run(const typename OxBlk<U>::T &z, const OxL &L, const OxCell &c, int d, int umax,
                                       int ty2, int ctb, float outer, float &g, float &sp, float &gs, float &sps,
                                       int r) {
    if constexpr (U < 0) {
    } else if constexpr (U <= 5) {
        if (!ADX_SMALL_R0 || r == 0) z.run(L, c, d, umax, ty2, gs, sps);   // counted on phase 0 only
    } else {
        z.run(L, c, d, umax, ctb, outer, g, sp);
    }
}
__device__ __forceinline__ float quad_sum_f(float v) {   // sum over the 4 lanes of a quad, in every lane
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));   // [1,0,3,2]
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));   // [2,3,0,1]
}

#ifdef ADX_STAMP
#define OX_STP_PARAMS , unsigned long long *st_acc, unsigned long long &st_last
#define OX_STP_ARGS , st_acc, st_last
#else
#define OX_STP_PARAMS
#define OX_STP_ARGS
#endif

// B: the interior-loop gather of every diagonal for one block of loop sizes
// (-1 = none), the block's shape factors held in registers for the whole sweep;
// four lanes per inner cell (16 cells per lane-set; OxSizeQ), one barrier per
// diagonal, as the M / F waves.
// wid: the wave as a compile-time constant (std::integral_constant; round 6), so
// the role fin(d, wid) runs on this wave is resolved per instance
template <int NSETS, int U0, int U1, int U2, int U3, int U4, class Fin, class Wid>
__device__ __forceinline__ void b_sweep(const OxL &L, int N, int lane, Wid wid, const Fin &fin OX_STP_PARAMS) {
    constexpr auto tb = [](int u) { return u >= 2 && u <= 4; };
    constexpr bool TB = tb(U0) || tb(U1) || tb(U2) || tb(U3) || tb(U4);
    constexpr bool H5 = U0 == 5 || U1 == 5 || U2 == 5 || U3 == 5 || U4 == 5;   // 2x3 loops (m23)
    const int r = lane & 3, cq = lane >> 2;
    typename OxBlk<U0>::T s0;
    typename OxBlk<U1>::T s1;
    typename OxBlk<U2>::T s2;
    typename OxBlk<U3>::T s3;
    typename OxBlk<U4>::T s4;
    ox_load<U0>(s0, L, r);
    ox_load<U1>(s1, L, r);
    ox_load<U2>(s2, L, r);
    ox_load<U3>(s3, L, r);
    ox_load<U4>(s4, L, r);
    const int ctb = r < 2 ? CT_BUL : CT_ONEN;   // the lane's special-shape outer factor table
    const float eTAU = L.ct[CT_FSM + 6];
    for (int d = N - 1; d >= 3; d--) {
        const int par = d & 1;
        const int umax = min(30, N - 3 - d);                      // outer spans d+2 .. d+2+umax
        // lanes = the pairable cells of diagonal d, compacted (records one step ahead)
        const int ncell = (d >= 4 && umax >= 0) ? uni(L.rcnt[par]) : 0;
        for (int c0 = 0; c0 < ncell; c0 += WAVE / 4) {
            const int idx = c0 + cq;   // the lane's cell (records: set idx / 64, lane idx % 64)
            const float *rr = L.rec + ((par * NSETS + (idx >> 6)) * OX_RF) * WAVE + (idx & (WAVE - 1));
            // word: i | ty2 << 8 | real << 16; a block reads only the fields its sizes use
            const int tp = __float_as_int(rr[0]);
            const int i = tp & 255;
            OxCell c;
            c.i = i;
            const int ty2 = (tp >> 8) & 255;
            c.mmin = rr[WAVE];
            c.tau_in = ty2 > 2 ? eTAU : 1.f;
            c.mo_in = rr[2 * WAVE];
            c.m23_in = H5 ? rr[3 * WAVE] : 0.f;
            c.t11 = c.t12 = c.t21 = c.t22 = 0.f;
            if constexpr (TB) {
                c.t11 = rr[4 * WAVE];
                c.t12 = rr[5 * WAVE];
                c.t21 = rr[6 * WAVE];
                c.t22 = rr[7 * WAVE];
            }
            const float outer = r < 2 ? c.tau_in : c.mo_in;
            float g = 0.f, sp = 0.f, gs = 0.f, sps = 0.f;
            OSTAMP(2);   // B cell setup
            ox_run<U0>(s0, L, c, d, umax, ty2, ctb, outer, g, sp, gs, sps, r);
            ox_run<U1>(s1, L, c, d, umax, ty2, ctb, outer, g, sp, gs, sps, r);
            ox_run<U2>(s2, L, c, d, umax, ty2, ctb, outer, g, sp, gs, sps, r);
            ox_run<U3>(s3, L, c, d, umax, ty2, ctb, outer, g, sp, gs, sps, r);
            ox_run<U4>(s4, L, c, d, umax, ty2, ctb, outer, g, sp, gs, sps, r);
            OSTAMP(3);   // B shapes
            // small sizes count once (phase 0), then the cell's total over its four lanes
            const float part = quad_sum_f(fmaf(g, c.mmin, sp) + (r == 0 ? fmaf(gs, c.mmin, sps) : 0.f));
            if (r == 0 && idx < ncell && (tp >> 16))   // the cell's natural slot (F reads lane = cell)
                L.part[((par * NSETS + ((i - 1) >> 6)) * OX_NB + wid) * WAVE + ((i - 1) & (WAVE - 1))] = part;
        }
        fin(d, wid);   // F of diagonal d + 1 on waves 0 and 1
        OSTAMP(5);
        lds_barrier();
        OSTAMP(6);   // barrier
    }
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

}  // namespace
}  // namespace adx
