// gfx950 McCaskill inside pass (the reference's scoring path, vrna_pf at
// scoring.cc:58,65; BASELINE configs 3-5 and the PF bench) with lanes = cells
// -- the same recursions, constraints, ligand motif and incremental folds as
// kernels.hip pf_group<…, 2, SumProd> (oracle/fold.c orc_pf_energy), mapped
// the way outside_cells.hip maps the outside pass:
//
//   * one workgroup (14 waves) per (walker, group of the apo and holo
//     variants of one (context, macrostate)), the two folds in lockstep as
//     float2 (ds_read_b64, v_pk_fma_f32: one instruction serves both);
//   * one anti-diagonal per step, ONE barrier per step.  Step s runs
//       B   the interior-loop sums of diagonal s (waves 0-6, loop sizes in
//           blocks of equal cost; four lanes per changed pairable cell, each
//           taking a quarter of a size's shapes; every shape one read of the
//           inner cell at a per-lane base plus an immediate offset);
//       M   the qm (fML) items of span s-2 (waves 10-13; K lanes per item so
//           that the few long items of late spans spread over the waves, the
//           split points read from the row-major qm and column-major qm1 at
//           immediate offsets);
//       F   the cells of diagonal s-1 (wave 7): qb, qbm, qm1;
//       Q   q5[s-1] (wave 8);
//       R   the setup records of diagonal s+1 (wave 9), built in four
//           stages a step apart.
//
// Covered: N <= 100 (LDS); longer folds take kernels.hip score_kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

#ifndef PX_NMW_CFG
#define PX_NMW_CFG 4
#endif
#ifndef PX_NB_CFG
#define PX_NB_CFG 8   // eight interior-loop waves (round 6: +1.2 % PF over seven, A/B r06f)
#endif
constexpr int PX_NB = PX_NB_CFG;      // interior-loop blocks (waves 0 .. PX_NB - 1)
constexpr int PX_NMW = PX_NMW_CFG;    // qm item waves (PX_NB + 3 .. PX_NB + 2 + PX_NMW)
constexpr int PX_M0 = PX_NB + 3;
constexpr int PX_NW = PX_M0 + PX_NMW;
constexpr int PX_NT = PX_NW * WAVE;
// Roles of the waves after the blocks (F, Q, R, then four qm waves: the qm wave
// with the most items sets the step at a power-of-two lane split, so a fourth
// qm wave halves it at about half of the spans; measured +1 % over 8 + 3).
constexpr int PX_WF = PX_NB, PX_WQ = PX_NB + 1, PX_WR = PX_NB + 2;   // F, Q, R
__host__ __device__ constexpr int px_mw(int w) {   // M wave index (0 = most items) or -1
    return w == PX_M0 ? 0 : w == PX_M0 + 1 ? 1 : w == PX_M0 + 3 ? 2 : w == PX_M0 + 2 ? 3
         : (w >= PX_M0 + 4 && w < PX_NW) ? w - PX_M0 : -1;
}
constexpr int PX_NMAX = 100;
#ifndef PX_PART
#define PX_PART 8   // interior-loop size partition of the eight blocks (pf_cells_kernel; 0: before r07g, A/B r07g-r07i)
#endif
#ifndef PX_ROLE_PRIO
#define PX_ROLE_PRIO 2   // s_setprio of the role waves (M, F, Q, R) over the interior-loop waves
#endif
constexpr int PX_RF = 8;              // record fields (rec_store): word, mmo, mo, m23, 1x1..2x2 factors
constexpr int PX_SLACK = 16;

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 sp2(float x) { return f2{x, x}; }
__device__ __forceinline__ bool is_mark2(f2 v) { return __float_as_uint(v.x) == 0x80000000u; }
// sum of v over the wave, both components (permlane32 swap folds x into lanes
// 0-31 and y into 32-63, one DPP chain finishes both; VALU only)
__device__ __forceinline__ f2 wave_sum_f2(f2 v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v.x), __float_as_uint(v.y), false, false);
    // lanes 0-31: x(l) + x(l+32); lanes 32-63: y(l-32) + y(l)
    float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0xb1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
    t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x4e, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
    t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x114, 0xf, 0xf, false));  // row_shr:4
    t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x118, 0xf, 0xf, false));  // row_shr:8
    t += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(t), 0x142, 0xa, 0xf, false));  // row_bcast:15
    return f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 31)),
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 63))};
}
// v + (v of the lane DPP control CTRL selects; 0 where it selects none)
template <int CTRL>
__device__ __forceinline__ f2 dpp_add2(f2 v) {
    const float x = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.x), CTRL, 0xf, 0xf, false));
    const float y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v.y), CTRL, 0xf, 0xf, false));
    return v + f2{x, y};
}

struct PxLay {
    int C, NP;
    size_t QB, QM, Q1, CC, PART, REC, CL, MLA, UC, Q5, CT, DT, PW, BY, MT, FL, BYTES;
    __host__ __device__ static size_t a16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ explicit PxLay(int N) {
        C = ((N - 4) * (N - 3)) / 2;
        NP = N + 2;
        size_t o = 0;
        QB = o;   o += a16((size_t(C) + PX_SLACK) * 8);           // qb * mismatchI(inner), diagonal-major
        QM = o;   o += a16((size_t(C) + PX_SLACK) * 8);           // qm, row-major
        Q1 = o;   o += a16((size_t(C) + PX_SLACK) * 8);           // qm1, column-major
        CC = o;   o += a16(size_t(C) + PX_SLACK);                 // inner-pair code per cell
        PART = o; o += a16(size_t(2) * 2 * PX_NB * WAVE * 8);     // [parity][lane-set][block][lane]
        REC = o;  o += a16(size_t(3) * 2 * PX_RF * WAVE * 4 + 16); // [diagonal % 3][set][field][lane]; counts
        CL = o;   o += a16(size_t(C) + size_t(NP));               // rank lists of the changed pairable cells + counts
        MLA = o;  o += a16(size_t(2) * NP * 8);                   // split part of qm, by span parity
        UC = o;   o += a16(size_t(2) * NP * 8);                   // unpaired part U(i, j) of qm by column j, by span parity
        Q5 = o;   o += a16(size_t(NP) * 8);
        CT = o;   o += a16(size_t(CT_SIZE) * 4);
        DT = o;   o += a16(size_t(DT_HP) * 4);                    // (hairpin lengths: XS->hp, scalar loads)
        PW = o;   o += a16(size_t(N + 9) * 4);                    // (expMLbase sigma)^t
        BY = o;   o += a16(size_t(7) * NP);                       // S, up, dn, ptn, enc, flg, mat
        MT = o;   o += a16(size_t(MAX_SPECIAL_HP) * 8 + 2 * MAX_MOTIF);   // special hairpins, motif codes / partners
        FL = o;   o += 16;                                        // block_or word
        BYTES = o;
    }
};

struct PxL {
    f2 *qb, *qm, *q1, *part, *mla, *uc, *q5;
    float *rec, *ct, *dt, *pw;
    int *rcnt;
    uint8_t *cc, *cl, *cn, *S, *up, *dn, *ptn, *enc, *flg, *mat;
    int N, NP;
};

__device__ __forceinline__ bool px_allowed(const PxL &L, int i, int j) {   // kernels.hip allowed()
    const int fi = L.flg[i], fj = L.flg[j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[i], pj = L.ptn[j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[i] == L.enc[j];
}

// interior-loop shape kinds (dev_types.hpp TermKind; -1 = generic)
__host__ __device__ constexpr int pkind(int n1, int n2) {
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
// constant factor of shape (u, n1) (adx_api.cpp addS / fgen); dz = 0 in every
// lane but not provably uniform, so the factors of a B wave's sizes live in
// VGPRs (as SGPRs they spill to lane slots, one v_readlane per use)
__device__ __forceinline__ float shape_factor(const DevScaled *XS, int u, int n1, int dz) {
    const int kd = pkind(n1, u - n1);
    const float *p = kd < 0 ? XS->fgen + (u - 6) * FG_ROW + n1 - 2
                   : kd == TK_STK ? XS->ctab + CT_FSM + 0
                   : kd == TK_B1 ? XS->ctab + CT_FSM + 1
                   : kd == TK_BUL ? XS->ctab + CT_FB + u
                   : kd == TK_1N ? XS->ctab + CT_F1N + u - 1
                   : kd == TK_I11 ? XS->ctab + CT_FSM + 2
                   : kd == TK_I22 ? XS->ctab + CT_FSM + 4
                   : kd == TK_M23 ? XS->ctab + CT_FSM + 5
                   : XS->ctab + CT_FSM + 3;
    return p[dz];
}

struct PxCell {              // per lane: the closing pair (i, i+s)
    int i, ty8, A, B;
    float tau, mo, m23;
    float t11, t12, t21, t22;
};

// One shape (N1, U - N1): the inner cell (i+1+N1, j-1-U+N1) on diagonal s-2-U
// at qb / cc row base + N1 (qb + o, cc + o: this lane's bases).
template <int U, int N1, bool MK>
__device__ __forceinline__ void pshape1(const PxL &L, const PxCell &c, const float *fv, const f2 *qb,
                                        const uint8_t *cc, uint32_t bits, f2 &g, f2 &sp) {
    constexpr int k = pkind(N1, U - N1);
    constexpr int FI = N1 < U - N1 ? N1 : U - N1;
    f2 v = qb[N1];
    // constrained cell: shapes past its unpaired runs count 0 (bit N1 of the size's
    // allowed-n1 mask as a factor: a compare-select becomes a branch around the load)
    if constexpr (MK) v *= sp2(float((bits >> N1) & 1u));
    if constexpr (k < 0) {
        g.x = fmaf(v.x, fv[FI], g.x);   // scalar FMAs: a packed one wants the factor duplicated in a register pair
        g.y = fmaf(v.y, fv[FI], g.y);
    } else {
        const float *ct = L.ct;
        const int ci = cc[N1];
        float f;
        if constexpr (k == TK_STK || k == TK_B1) {
            f = ct[CT_INVMM + ci] * ct[CT_STK + c.ty8 + ((ci * 41) >> 10)] * fv[FI];
        } else if constexpr (k == TK_BUL) {
            f = ct[CT_BUL + ci] * (c.tau * fv[FI]);
        } else if constexpr (k == TK_1N) {
            f = ct[CT_ONEN + ci] * (c.mo * fv[FI]);
        } else if constexpr (k == TK_M23) {
            f = ct[CT_INVMM + ci] * ct[CT_M23O + ci] * (c.m23 * fv[FI]);
        } else {
            const float tv = k == TK_I11 ? c.t11 : k == TK_I12 ? c.t12 : k == TK_I21 ? c.t21 : c.t22;
            f = ct[CT_INVMM + ci] * (tv * fv[FI]);
        }
        sp = fma2(v, sp2(f), sp);
    }
}
template <int U, bool MK, int... N1s>
__device__ __forceinline__ void pshape_seq(std::integer_sequence<int, N1s...>, const PxL &L, const PxCell &c,
                                           const float *fv, const f2 *qb, const uint8_t *cc, uint32_t bits, f2 &g,
                                           f2 &sp) {
    (pshape1<U, N1s, MK>(L, c, fv, qb, cc, bits, g, sp), ...);
}
// every shape factor is symmetric in (n1, n2) (adx_api.cpp build_scaled): a
// size keeps U/2 + 1 of them, shape n1 reads fv[min(n1, U - n1)]
template <int U>
struct PxSize {
    float fv[U < 0 ? 1 : U / 2 + 1];
    __device__ __forceinline__ void load(const DevScaled *XS, int dz) {
        if constexpr (U >= 0)
#pragma unroll
            for (int n1 = 0; n1 <= U / 2; n1++) fv[n1] = shape_factor(XS, U, n1, dz);
    }
    template <bool MK>
    __device__ __forceinline__ void run(const PxL &L, const PxCell &c, int s, int umax, f2 &g, f2 &sp) const {
        if constexpr (U >= 0) {
            if (U <= umax) {
                const int o = off(s - 2 - U, L.N) + c.i;   // inner cell (i+1+n1, ...) at o + n1
                uint32_t bits = 0;
                if constexpr (MK) {   // n1 <= A and U - n1 <= B
                    const int lo = max(0, U - c.B), hi = min(U, c.A);
                    bits = hi < lo ? 0u : ((2u << hi) - 1u) & ~((1u << lo) - 1u);
                }
                pshape_seq<U, MK>(std::make_integer_sequence<int, U + 1>{}, L, c, fv, L.qb + o, L.cc + o, bits, g,
                                  sp);
            }
        }
    }
};

// Loop size U >= 6 over the four lanes of a cell (phase r = lane & 3): lane r
// takes one of the four special shapes -- bulges (0,U) (U,0), 1 x n loops
// (1,U-1) (U-1,1) -- and the generic shapes n1 = 2 + r, 6 + r, ... <= U - 2
// (one read at a per-lane base + immediate offset 4m, its factor in a VGPR;
// 0 past the size, so the last round needs no mask).  Every lane runs the same
// code; the four lanes' sums are added in a fixed order (bit-identical refolds).
template <int U>
struct PxSizeQ {
    static constexpr int NR = U >= 6 ? (U - 3 + 3) / 4 : 1;   // generic rounds
    float gf[NR];
    float fsp;      // the lane's special-shape factor (bulge FB[U] or 1 x n F1N[U-1])
    int n1sp;       // the lane's special shape
    __device__ __forceinline__ void load(const DevScaled *XS, int r) {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const int n1 = 2 + 4 * m + r;
            gf[m] = n1 <= U - 2 ? XS->fgen[(U - 6) * FG_ROW + n1 - 2] : 0.f;
        }
        n1sp = r == 0 ? 0 : r == 1 ? U : r == 2 ? 1 : U - 1;
        fsp = r < 2 ? XS->ctab[CT_FB + U] : XS->ctab[CT_F1N + U - 1];
    }
    template <bool MK>
    __device__ __forceinline__ void run(const PxL &L, const PxCell &c, int s, int umax, int r, int ctb, float outer,
                                        f2 &g, f2 &sp) const {
        if (U <= umax) {
            const int o = off(s - 2 - U, L.N) + c.i;   // inner cell (i+1+n1, ...) at o + n1
            uint32_t bits = ~0u;
            if constexpr (MK) {   // n1 <= A and U - n1 <= B
                const int lo = max(0, U - c.B), hi = min(U, c.A);
                bits = hi < lo ? 0u : ((2u << hi) - 1u) & ~((1u << lo) - 1u);
            }
            // special shape of this lane
            {
                f2 v = L.qb[o + n1sp];
                if constexpr (MK) v *= sp2(float((bits >> n1sp) & 1u));
                const int ci = L.cc[o + n1sp];
                sp = fma2(v, sp2(L.ct[ctb + ci] * (outer * fsp)), sp);
            }
            // generic shapes n1 = 2 + r + 4m
            const f2 *q = L.qb + o + 2 + r;
            const uint32_t bm = bits >> (2 + r);
#pragma unroll
            for (int m = 0; m < NR; m++) {
                f2 v = q[4 * m];
                if constexpr (MK) v *= sp2(float((bm >> (4 * m)) & 1u));
                g.x = fmaf(v.x, gf[m], g.x);
                g.y = fmaf(v.y, gf[m], g.y);
            }
        }
    }
};

#ifdef ADX_STAMP
__device__ unsigned long long g_stamps_p[16][12];
#define PSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#define PX_STP_PARAMS , unsigned long long *st_acc, unsigned long long &st_last
#define PX_STP_ARGS , st_acc, st_last
#else
#define PSTAMP(k) do { } while (0)
#define PX_STP_PARAMS
#define PX_STP_ARGS
#endif

// B: interior-loop sums of every diagonal for one block of loop sizes.  Lanes
// = (cell, phase r): four lanes per cell (16 cells per lane-set), sizes >= 6 as
// PxSizeQ (shapes spread over the phases), sizes <= 5 (the stack, 1x1..2x3
// table loops) computed whole by every lane and counted once (phase 0).  The
// four partials are summed by DPP and phase 0 writes the cell's natural slot.
#ifndef ADX_SMALL_R0
#define ADX_SMALL_R0 1   // sizes <= 5 on phase 0 only (the other phases' copies are discarded)
#endif
template <int U>
struct PxBlk {   // the size's state in a B wave
    using T = typename std::conditional<(U < 0), PxSize<-1>, typename std::conditional<(U <= 5), PxSize<U>, PxSizeQ<U>>::type>::type;
};
template <int U, bool MK>
__device__ __forceinline__ void px_run(const typename PxBlk<U>::T &z, const PxL &L, const PxCell &c, int s, int umax,
                                       int r, int ctb, float outer, f2 &g, f2 &sp, f2 &gs, f2 &sps) {
    if constexpr (U < 0) {
    } else if constexpr (U <= 5) {
        // counted on phase 0 only: the other phases skip the reads (LDS cycles)
        if (!ADX_SMALL_R0 || r == 0) z.template run<MK>(L, c, s, umax, gs, sps);
    } else {
        z.template run<MK>(L, c, s, umax, r, ctb, outer, g, sp);
    }
}
template <int U>
__device__ __forceinline__ void px_load(typename PxBlk<U>::T &z, const DevScaled *XS, int r) {
    if constexpr (U < 0) {
    } else if constexpr (U <= 5) {
        z.load(XS, 0);   // uniform factors: SGPRs
    } else {
        z.load(XS, r);
    }
}
__device__ __forceinline__ f2 quad_sum(f2 v) {   // sum over the 4 lanes of a quad, in every lane
    v = dpp_add2<0xb1>(v);   // quad_perm [1,0,3,2]
    return dpp_add2<0x4e>(v);   // quad_perm [2,3,0,1]
}

template <int U0, int U1, int U2, int U3, int U4>
__device__ __forceinline__ void pb_sweep(const PxL &L, const DevScaled *XS, int N, int lane, int wid,
                                         bool constrained, int s_end PX_STP_PARAMS) {
    constexpr auto tb = [](int u) { return u >= 2 && u <= 4; };
    constexpr bool TB = tb(U0) || tb(U1) || tb(U2) || tb(U3) || tb(U4);
    constexpr bool H5 = U0 == 5 || U1 == 5 || U2 == 5 || U3 == 5 || U4 == 5;   // 2x3 loops (m23)
    const float eTAU = XS->ctab[CT_FSM + 6];
    const int r = lane & 3, cq = lane >> 2;
    typename PxBlk<U0>::T s0;
    typename PxBlk<U1>::T s1;
    typename PxBlk<U2>::T s2;
    typename PxBlk<U3>::T s3;
    typename PxBlk<U4>::T s4;
    px_load<U0>(s0, XS, r);
    px_load<U1>(s1, XS, r);
    px_load<U2>(s2, XS, r);
    px_load<U3>(s3, XS, r);
    px_load<U4>(s4, XS, r);
    const int ctb = r < 2 ? CT_BUL : CT_ONEN;   // the lane's special-shape inner factor table
    // the first lane-set's records and the count of diagonal D, loaded a step
    // ahead (the record wave writes them two steps ahead, slot D % 3): issued
    // at the top of a step, they complete under its first reads
    struct Pre {
        int n, fl;
        float mmo, mo, m23, t11, t12, t21, t22;
    };
    auto pre_load = [&](int D) {
        Pre p;
        const int sl = D % 3;
        p.n = (D <= N - 1 && D >= 6) ? L.rcnt[sl] : 0;
        const float *rr = L.rec + (sl * 2 * PX_RF) * WAVE + cq;
        p.fl = __float_as_int(rr[0]);
        p.mmo = rr[WAVE];
        p.mo = rr[2 * WAVE];
        p.m23 = H5 ? rr[3 * WAVE] : 0.f;
        p.t11 = p.t12 = p.t21 = p.t22 = 0.f;
        if constexpr (TB) {
            p.t11 = rr[4 * WAVE];
            p.t12 = rr[5 * WAVE];
            p.t21 = rr[6 * WAVE];
            p.t22 = rr[7 * WAVE];
        }
        return p;
    };
    Pre cur = pre_load(4);
    for (int s = 4; s <= s_end; s++) {
        const int sl = s % 3;
        const Pre nxt = pre_load(s + 1);
        const int umax = min(30, s - 6);   // no interior loop fits a span below 6
        const int ncell = (s <= N - 1 && umax >= 0) ? uni(cur.n) : 0;
        for (int c0 = 0; c0 < ncell; c0 += WAVE / 4) {
            const int idx = c0 + cq;   // the lane's cell (records: set idx / 64, lane idx % 64)
            // word: i | ty << 7 | A << 10 | B << 18 | masked << 26 | real << 27; a block
            // reads only the fields its sizes use
            Pre q = cur;
            if (c0 > 0) {
                const float *rr = L.rec + ((sl * 2 + (idx >> 6)) * PX_RF) * WAVE + (idx & (WAVE - 1));
                q.fl = __float_as_int(rr[0]);
                q.mmo = rr[WAVE];
                q.mo = rr[2 * WAVE];
                q.m23 = H5 ? rr[3 * WAVE] : 0.f;
                if constexpr (TB) {
                    q.t11 = rr[4 * WAVE];
                    q.t12 = rr[5 * WAVE];
                    q.t21 = rr[6 * WAVE];
                    q.t22 = rr[7 * WAVE];
                }
            }
            const int fl = q.fl;
            PxCell c;
            c.i = fl & 127;
            const int ty = (fl >> 7) & 7;
            c.ty8 = ty * 8;
            c.A = (fl >> 10) & 255;
            c.B = (fl >> 18) & 255;
            const float mmo = q.mmo;
            c.tau = ty > 2 ? eTAU : 1.f;
            c.mo = q.mo;
            c.m23 = q.m23;
            c.t11 = q.t11;
            c.t12 = q.t12;
            c.t21 = q.t21;
            c.t22 = q.t22;
            const float outer = r < 2 ? c.tau : c.mo;
            f2 g = {0.f, 0.f}, sp = {0.f, 0.f}, gs = {0.f, 0.f}, sps = {0.f, 0.f};
            PSTAMP(2);
            // shapes past a cell's allowed unpaired runs (constraints) are masked
            const bool mk = constrained && __ballot((fl >> 26) & 1) != 0;
            if (mk) {
                px_run<U0, true>(s0, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U1, true>(s1, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U2, true>(s2, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U3, true>(s3, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U4, true>(s4, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
            } else {
                px_run<U0, false>(s0, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U1, false>(s1, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U2, false>(s2, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U3, false>(s3, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                px_run<U4, false>(s4, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
            }
            PSTAMP(3);
            // small sizes count once (phase 0), then the cell's total over its four lanes
            const f2 part = quad_sum(fma2(g, sp2(mmo), sp) + (r == 0 ? fma2(gs, sp2(mmo), sps) : f2{0.f, 0.f}));
            if (r == 0 && idx < ncell && ((fl >> 27) & 1))
                L.part[(((s & 1) * 2 + ((c.i - 1) >> 6)) * PX_NB + wid) * WAVE + ((c.i - 1) & (WAVE - 1))] = part;
        }
        cur = nxt;
        PSTAMP(5);
        lds_barrier();
        PSTAMP(6);
    }
}

// One workgroup per (walker, group).  gout: [W][n_variants] ensemble energies
// (kcal/mol, as score_sequence writes dG), the scores follow in combine_kernel.
__global__ void __launch_bounds__(PX_NT, 1)
pf_cells_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, const int *mask,
                float *gout) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef ADX_STAMP
    unsigned long long st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    const int wb = blockIdx.x / ka.n_groups2, grp = blockIdx.x % ka.n_groups2;
    if (wb >= W) return;
    const WalkerRef wr = walker_ref(ka, mask, wb);   // heaviest refolds first
    if (!wr.on) return;
    const int w = wr.w;
    const int vs0 = ka.groups2[2 * grp], vs1 = ka.groups2[2 * grp + 1];
    const DevVariant V = ka.variants[vs0];
    const bool hol0 = ka.variants[vs0].motif != 0, hol1 = ka.variants[vs1].motif != 0;
    const int N = uni(V.N);
    const PxLay Y(N);
    PxL L;
    L.qb = reinterpret_cast<f2 *>(smem + Y.QB);
    L.qm = reinterpret_cast<f2 *>(smem + Y.QM);
    L.q1 = reinterpret_cast<f2 *>(smem + Y.Q1);
    L.cc = reinterpret_cast<uint8_t *>(smem + Y.CC);
    L.part = reinterpret_cast<f2 *>(smem + Y.PART);
    L.rec = reinterpret_cast<float *>(smem + Y.REC);
    L.rcnt = reinterpret_cast<int *>(smem + Y.REC + size_t(3) * 2 * PX_RF * WAVE * 4);
    L.cl = reinterpret_cast<uint8_t *>(smem + Y.CL);       // cl[off(D) + rank] = i
    L.cn = L.cl + Y.C;                                      // cn[D] = count
    L.mla = reinterpret_cast<f2 *>(smem + Y.MLA);
    L.uc = reinterpret_cast<f2 *>(smem + Y.UC);
    L.q5 = reinterpret_cast<f2 *>(smem + Y.Q5);
    L.ct = reinterpret_cast<float *>(smem + Y.CT);
    L.dt = reinterpret_cast<float *>(smem + Y.DT);
    L.pw = reinterpret_cast<float *>(smem + Y.PW);
    uint8_t *by = reinterpret_cast<uint8_t *>(smem + Y.BY);
    L.S = by;
    L.up = by + Y.NP;
    L.dn = by + 2 * Y.NP;
    L.ptn = by + 3 * Y.NP;
    L.enc = by + 4 * Y.NP;
    L.flg = by + 5 * Y.NP;
    L.mat = by + 6 * Y.NP;
    uint32_t *spk = reinterpret_cast<uint32_t *>(smem + Y.MT);   // special-hairpin keys (padded: no match)
    float *spv = reinterpret_cast<float *>(smem + Y.MT + MAX_SPECIAL_HP * 4);
    uint8_t *mcode = reinterpret_cast<uint8_t *>(smem + Y.MT + MAX_SPECIAL_HP * 8);
    int8_t *mpt = reinterpret_cast<int8_t *>(mcode + MAX_MOTIF);
    L.N = N;
    L.NP = Y.NP;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
    const int C = Y.C, NP = Y.NP;
    const DevTables &T = *ka.T;

    // ---- incremental fold state (kernels.hip score_sequence / Inc): this group's
    // tables of the current sequence (src) and the proposal's (dst)
    const size_t Cs = size_t(ka.cells), B1 = 3 * Cs + size_t(ka.Nmax) + 2;
    const float *src = nullptr;
    float *dst = nullptr;
    const uint4 *cc_src = nullptr;   // the slots' per-cell codes (dev_types.hpp inc_cc_offset_pf)
    uint4 *cc_dst = nullptr;
    int m_lo = 0, m_hi = 0;
    if (ka.tab) {
        const int cur = wr.cur;
        float *base = ka.tab + size_t(w) * 2 * ka.tab_slot;
        dst = base + size_t(1 - cur) * ka.tab_slot + size_t(grp) * 2 * B1;
        const size_t cco = inc_cc_offset_pf(ka.cells, ka.Nmax, ka.n_groups2, grp);
        cc_dst = reinterpret_cast<uint4 *>(base + size_t(1 - cur) * ka.tab_slot + cco);
        if (wr.valid && wr.c0 >= 0) {
            src = base + size_t(cur) * ka.tab_slot + size_t(grp) * 2 * B1;
            cc_src = reinterpret_cast<const uint4 *>(base + size_t(cur) * ka.tab_slot + cco);
            m_lo = wr.c0 + 1 + V.before_len;
            m_hi = wr.c1 + 1 + V.before_len;
        }
    }
    const bool incr = src != nullptr;
    if (tid == 0) *reinterpret_cast<int *>(smem + Y.FL) = 0;   // block_or word (read after two barriers)
    m_lo = uni(m_lo);
    m_hi = uni(m_hi);
    auto clo = [&](int D) { return incr ? max(1, m_lo - 1 - D) : 1; };
    auto chi = [&](int D) { return incr ? min(N - D, m_hi + 1) : N - D; };
    auto qlo = [&](int sq) { return incr ? max(1, m_lo - 2 - sq) : 1; };
    auto qhi = [&](int sq) { return incr ? min(N - sq, m_hi + 2) : N - sq; };

    PSTAMP(8);   // the prologue (walker, slot, variant words)
    // ---- setup loads (round 6): the one element of every table and of the sequence /
    // constraint arrays this thread stores, all in flight at once and stored before
    // the restore's loads are issued (a loop per table waited on each load in turn, the
    // first behind the restore's: ~14k cycles per group, stamps r06p "tables")
    static_assert(CT_SIZE <= PX_NT && 288 <= PX_NT && PX_NMAX + 9 <= PX_NT && MAX_SPECIAL_HP <= PX_NT &&
                  MAX_MOTIF <= PX_NT && PX_NMAX + 2 <= PX_NT, "one setup element per thread");
    const float v_ct = XS->ctab[min(tid, CT_SIZE - 1)];
    const float v_mh = (&T.mmH[0][0][0])[min(tid, 199)], v_mi = (&T.mmI[0][0][0])[min(tid, 199)],
                v_ms = (&T.mlstem[0][0][0])[min(tid, 199)];
    const float v_ex = (&T.ext[0][0][0])[min(tid, 287)], v_tau = T.termAU[tid & 7];
    const float v_pw = XS->pwml[min(tid, N + 8)];
    const int n_sp = XS->n_special;
    const uint32_t v_spk = XS->sp_key[min(tid, MAX_SPECIAL_HP - 1)];
    const float v_spv = XS->sp_val[min(tid, MAX_SPECIAL_HP - 1)];
    const uint8_t v_mc = XS->motif_code[min(tid, MAX_MOTIF - 1)];
    const int8_t v_mp = XS->motif_pt[min(tid, MAX_MOTIF - 1)];
    // hairpin length factors of this wave's per-cell-pass diagonals D = 4 + wid + NW m (lane m)
    static_assert(4 + (WAVE - 1) * PX_NW > PX_NMAX, "hpl covers every diagonal");
    const float hpl = XS->hp[min(3 + wid + PX_NW * lane, NMAX)];
    const uint8_t *cons = ka.cons + V.cons_off;
    const int kp = min(tid, NP - 1);   // this thread's position
    uint8_t v_s, v_up, v_dn, v_pt, v_en, v_fl;
    {
        const uint8_t *bef = nullptr, *aft = nullptr;
        int blen = 0;
        if (V.ctx >= 0) {
            bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
            blen = ka.ctx_off[4 * V.ctx + 1];
            aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
        }
        const uint8_t *raw = seqs + size_t(w) * ka.Nraw;
        const int pp = kp >= 1 && kp <= N ? kp - 1 : blen;   // outside 1..N: a valid byte, discarded
        const uint8_t *sp = pp < blen ? bef + pp : (pp < blen + ka.Nraw ? raw + (pp - blen) : aft + (pp - blen - ka.Nraw));
        v_s = *sp;
        v_up = cons[kp];
        v_dn = cons[NP + kp];
        v_pt = cons[2 * NP + kp];
        v_en = cons[3 * NP + kp];
        v_fl = cons[4 * NP + kp];
    }

    // ---- sequence, constraint arrays, tables (kernels.hip pf_group setup): the stores
    if (tid < NP) {
        L.S[tid] = (tid >= 1 && tid <= N) ? v_s : 0;
        L.up[tid] = v_up;
        L.dn[tid] = v_dn;
        L.ptn[tid] = v_pt;
        L.enc[tid] = v_en;
        L.flg[tid] = v_fl;
        L.mat[tid] = 0;
    }
    const bool cst = tid >= 1 && tid <= N && (v_fl | v_pt) != 0;
    if (tid < CT_SIZE) L.ct[tid] = v_ct;
    if (tid < 200) {
        L.dt[DT_MMH + tid] = v_mh;
        L.dt[DT_MMI + tid] = v_mi;
        L.dt[DT_MLS + tid] = v_ms;
    }
    if (tid < 288) L.dt[DT_EXT + tid] = v_ex;
    if (tid < 8) L.dt[DT_TAU + tid] = v_tau;
    if (tid < N + 9) L.pw[tid] = v_pw;
    if (tid < MAX_SPECIAL_HP) {
        const bool on = tid < n_sp;
        spk[tid] = on ? v_spk : 0xFFFFFFFFu;   // hp_key never sets the top bits
        spv[tid] = on ? v_spv : 0.f;
    }
    if (tid < MAX_MOTIF) {
        mcode[tid] = v_mc;
        mpt[tid] = v_mp;
    }
    PSTAMP(9);   // setup loads and stores
    // ---- refold restore: every table from the current slot (the changed cells are
    // recomputed over it), two cells per lane and load, both folds interleaved.
    // The loads are issued here and stored to LDS after the motif scan, so their
    // HBM latency overlaps the rest of the setup.  (HBM side dword-aligned only
    // when cells or B1 are odd: fine for global loads.)
    constexpr int RS = 8;   // loads per lane: 3 * C / 2 <= RS * PX_NT for N <= PX_NMAX
    static_assert(3 * (((PX_NMAX - 4) * (PX_NMAX - 3) / 2) / 2) <= RS * PX_NT, "restore loads fit RS per lane");
    const int half = C >> 1;
    float2 rsx[RS], rsy[RS];
    const int C16 = (C + 15) >> 4;
    static_assert(((PX_NMAX - 4) * (PX_NMAX - 3) / 2 + 15) / 16 <= PX_NT, "one code load per thread");
    uint4 rcv = make_uint4(0, 0, 0, 0);
    f2 rod = f2{0.f, 0.f}, r5 = f2{0.f, 0.f};
    if (incr) {
#pragma unroll
        for (int t = 0; t < RS; t++) {
            const int k = tid + t * PX_NT;
            const int kk = k < 3 * half ? k : 0;
            const int a = kk / half, c = kk - a * half;
            const float *sa = src + a * Cs + 2 * c;
            rsx[t] = *reinterpret_cast<const float2 *>(sa);
            rsy[t] = *reinterpret_cast<const float2 *>(sa + B1);
        }
        rcv = cc_src[tid < C16 ? tid : 0];   // the codes (round 6: the band's are recomputed)
        const int ko = min(tid, 2);           // the odd last cell of each table, q5's prefix
        rod = f2{src[ko * Cs + max(C - 1, 0)], src[B1 + ko * Cs + max(C - 1, 0)]};
        const int k5 = min(tid, N);
        r5 = f2{src[3 * Cs + k5], src[B1 + 3 * Cs + k5]};
    } else {
        for (int k = tid; k < C; k += PX_NT) L.qm[k] = f2{0.f, 0.f};   // spans N-2, N-1 are never computed
    }
    for (int k = tid; k < 2 * NP; k += PX_NT) L.mla[k] = f2{0.f, 0.f};
    for (int k = C + tid; k < C + PX_SLACK; k += PX_NT) L.qb[k] = L.qm[k] = L.q1[k] = f2{0.f, 0.f};
    PSTAMP(10);   // the restore's loads issued
    __syncthreads();   // orders tid 0's zeroing of the block_or word before the ORs
    const bool constrained = block_or(reinterpret_cast<int *>(smem + Y.FL), cst);
    PSTAMP(1);
    if (tid == 0) {   // ViennaRNA's S1 wrap-around
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
    }
    const int mL = XS->motif_len;
    const bool any_motif = (hol0 || hol1) && mL > 0;
    __syncthreads();
    if (any_motif) {
        // motif sites: the sequence (one lane per start), then the constraints of
        // each matching start (one wave per start, lanes = motif positions)
        for (int o = tid + 1; o + mL - 1 <= N; o += PX_NT) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) ok = L.S[o + k] == mcode[k];
            L.mat[o] = ok ? 1 : 0;
        }
        __syncthreads();
        for (int o = 1 + wid; o + mL - 1 <= N; o += PX_NW) {
            if (!uni(L.mat[o])) continue;
            bool ok = true;
            for (int k = lane; k < mL; k += WAVE) {
                const int pk = mpt[k];
                if (pk < 0) ok = ok && L.up[o + k] >= 1;
                else if (pk > k) ok = ok && px_allowed(L, o + k, o + pk);
            }
            const bool all = __ballot(!ok) == 0;
            if (lane == 0) L.mat[o] = all ? 1 : 0;
        }
    }
    if (incr) {   // the restore's stores (loads issued at the start)
        float4 *qd = reinterpret_cast<float4 *>(L.qb);   // qb, qm, q1 contiguous at a16(C + slack) strides
        const size_t ls4 = (Y.QM - Y.QB) >> 4;
#pragma unroll
        for (int t = 0; t < RS; t++) {
            const int k = tid + t * PX_NT;
            if (k < 3 * half) {
                const int a = k / half, c = k - a * half;
                qd[a * ls4 + c] = float4{rsx[t].x, rsy[t].x, rsx[t].y, rsy[t].y};
            }
        }
        if ((C & 1) && tid < 3) L.qb[tid * (ls4 * 2) + C - 1] = rod;
        if (tid < C16) reinterpret_cast<uint4 *>(L.cc)[tid] = rcv;
        static_assert(PX_NMAX < PX_NT, "one q5 entry per thread");
        if (tid <= m_lo - 2 && tid <= N) L.q5[tid] = r5;
    }
    __syncthreads();
    PSTAMP(7);   // motif sites + the restore's stores (the wait for its loads)
    const uint8_t *S = L.S;
    const float *ct = L.ct;
    const float sig1 = XS->sig[1], mlbase_sig = XS->mlbase_sig, mlclosing = XS->mlclosing;
    const float mext = XS->motif_extra;
    const int nsp = XS->n_special < MAX_SPECIAL_HP ? XS->n_special : MAX_SPECIAL_HP;

    // cells by diagonal (wave w: diagonals 4 + w, 4 + w + NW, ...; lanes = i): the
    // inner code of every cell; the changed cells' hairpin (+ motif) initial value
    // (pairable) or the mark, and multiloop stem in qm1 (F reads both before it
    // overwrites them) -- in a refold every other cell was restored above; and the
    // rank list of the changed pairable cells (the B lanes): cl[off(D) + rank] = i,
    // cn[D] = count
    for (int D = 4 + wid; D <= N - 1; D += PX_NW) {
        const int od = off(D, N), lo = clo(D), hi = chi(D);
        int base = 0;
        // a refold's band rows only (round 6: the other cells' codes are restored)
        for (int i0 = lo; i0 <= hi; i0 += WAVE) {
            const int i = i0 + lane;
            const bool cell = i <= hi;
            const bool inb = cell && i >= lo && i <= hi;
            bool pr = false;
            if (cell) {
                const int j = i + D;
                const int type = ptype(S[i], S[j]);
                L.cc[od + i - 1] = uint8_t(rtype(type) * 25 + S[j + 1] * 5 + S[i - 1]);
                if (inb) {
                    pr = type != 0 && px_allowed(L, i, j);
                    f2 init = f2{-0.f, -0.f};
                    float m1 = 0.f;
                    if (pr) {
                        const int u = D - 1;
                        float h = 0.f;
                        if (L.up[i + 1] >= u) {
                            bool special = false;
                            if (u == 3 || u == 4 || u == 6) {
                                const int sh = special_hp(spk, hp_key(S, i, u + 2));
                                if (sh >= 0) {
                                    h = spv[sh];
                                    special = true;
                                }
                            }
                            if (!special)
                                h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hpl), (D - 4 - wid) / PX_NW)) * ((u == 3) ? L.dt[DT_TAU + type]
                                                                : L.dt[DT_MMH + type * 25 + S[i + 1] * 5 + S[j - 1]]);
                        }
                        const bool mx = D == mL - 1 && mL > 0 && L.mat[i];
                        init = f2{(mx && hol0) ? h + mext : h, (mx && hol1) ? h + mext : h};
                        m1 = L.dt[DT_MLS + type * 25 + S[i - 1] * 5 + S[j + 1]];
                    }
                    L.qb[od + i - 1] = init;
                    L.q1[colb(j) + i - 1] = f2{m1, m1};
                }
            }
            const uint64_t m = __ballot(pr);
            const int slot = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
            if (pr) L.cl[od + slot] = uint8_t(i);
            base += __popcll(m);
        }
        if (lane == 0) L.cn[D] = uint8_t(base);
    }
    for (int k = tid; k <= 3 && k <= N; k += PX_NT) {   // q5[0..3] (pf_group: unpaired prefix)
        float q = 1.f;
        bool ok = true;
        for (int t = 1; t <= k; t++) {
            ok = ok && L.up[t] >= 1;
            q *= sig1;
        }
        L.q5[k] = ok ? f2{q, q} : f2{0.f, 0.f};
    }
    __syncthreads();
    PSTAMP(0);

    // ---- records (wave 9): the changed pairable cells of diagonal D (rank
    // lists) and their setup values -- outer factors of the closing pair, the
    // unpaired runs, the 1x1..2x2 table factors (HBM/L2 loads) -- gathered at step
    // D - 2 (rec_load) and written at step D - 1 (rec_store), so the table loads
    // complete in the shadow of a step
    struct Pend {
        int n;                       // cells
        int w1[2];                   // per lane-set: the record word (pb_sweep)
        float mmo[2], mo[2], m23[2], t11[2], t12[2], t21[2], t22[2];
    };
    struct Seq {                     // per lane-set: i and the bases around the closing pair
        int n;
        int i[2], sq[2];             // sq: ty | si1 << 4 | sj1 << 8 | si2 << 12 | sj2 << 16 | A << 20 (A, B: 6 bits)
        int ab[2];                   // A | B << 8
    };
    // four stages a step apart, one LDS round trip each: idx_load (rank list),
    // seq_load (bases), rec_load (tables: LDS factors, HBM/L2 1x1..2x2
    // factors), rec_store
    struct Idx {                     // per lane-set: i of the lane's cell (the first cell on idle lanes)
        int n;
        int i[2];
    };
    auto idx_load = [&](int D) {
        Idx X;
        X.n = 0;
        X.i[0] = X.i[1] = 1;
        if (D < 6 || D > N - 1) return X;
        const int od = off(D, N);
        X.n = uni(L.cn[D]);
        const int i0 = L.cl[od];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int idx = k * WAVE + lane;
            const int ir = L.cl[od + min(idx, N - D - 1)];
            X.i[k] = idx < X.n ? ir : i0;
        }
        return X;
    };
    auto seq_load = [&](int D, const Idx &X) {
        Seq Q;
        Q.n = X.n;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (k * WAVE >= Q.n) break;
            const int i = X.i[k], j = i + D;
            Q.i[k] = i;
            Q.sq[k] = ptype(S[i], S[j]) | (S[i + 1] << 4) | (S[j - 1] << 8) | (S[i + 2] << 12) | (S[j - 2] << 16);
            Q.ab[k] = L.up[i + 1] | (L.dn[j - 1] << 8);
        }
        return Q;
    };
    auto rec_load = [&](int D, const Seq &Q) {
        Pend P;
        P.n = Q.n;
        const int umax = min(30, D - 6);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (k * WAVE >= Q.n) break;
            const bool v = k * WAVE + lane < Q.n;
            const int i = Q.i[k], sqk = Q.sq[k];
            const int ty = sqk & 15, si1 = (sqk >> 4) & 15, sj1 = (sqk >> 8) & 15, si2 = (sqk >> 12) & 15,
                      sj2 = (sqk >> 16) & 15;
            const int oc = ty * 25 + si1 * 5 + sj1;
            const int A = Q.ab[k] & 255, Bq = Q.ab[k] >> 8;
            P.t11[k] = P.t12[k] = P.t21[k] = P.t22[k] = 0.f;
            {   // kernels.hip load_chunk: the table factors of the 1x1..2x2 loops
                auto t2of = [&](int n1, int n2) { return (L.cc[off(D - 2 - n1 - n2, N) + i + n1] * 41) >> 10; };
                if (umax >= 2) P.t11[k] = T.int11[ty][t2of(1, 1)][si1][sj1];
                if (umax >= 3) {
                    P.t12[k] = T.int21[ty][t2of(1, 2)][si1][sj2][sj1];
                    P.t21[k] = T.int21[t2of(2, 1)][ty][sj1][si1][si2];
                }
                if (umax >= 4) P.t22[k] = T.int22[ty][t2of(2, 2)][si1][si2][sj2][sj1];
            }
            const bool mkc = A < umax || Bq < umax;
            P.w1[k] = i | (ty << 7) | (A << 10) | (Bq << 18) | (mkc ? (1 << 26) : 0) | (v ? (1 << 27) : 0);
            P.mmo[k] = L.dt[DT_MMI + oc];
            P.mo[k] = ct[CT_ONEN + oc] * P.mmo[k];
            P.m23[k] = ct[CT_M23O + oc];
        }
        return P;
    };
    auto rec_store = [&](int D, const Pend &P) {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (k * WAVE >= P.n) break;
            float *r = L.rec + (((D % 3) * 2 + k) * PX_RF) * WAVE + lane;
            r[0] = __int_as_float(P.w1[k]);
            r[WAVE] = P.mmo[k];
            r[2 * WAVE] = P.mo[k];
            r[3 * WAVE] = P.m23[k];
            r[4 * WAVE] = P.t11[k];
            r[5 * WAVE] = P.t12[k];
            r[6 * WAVE] = P.t21[k];
            r[7 * WAVE] = P.t22[k];
        }
        if (lane == 0) L.rcnt[D % 3] = P.n;
    };
    Pend pend;
    Seq seqp;
    Idx idxp;
    if (wid == PX_WR) {   // the records run two steps ahead of B (which loads them one step ahead)
        rec_store(4, rec_load(4, seq_load(4, idx_load(4))));   // the sweep's first B diagonals (no loop fits: count 0)
        rec_store(5, rec_load(5, seq_load(5, idx_load(5))));
        pend = rec_load(6, seq_load(6, idx_load(6)));
        seqp = seq_load(7, idx_load(7));
        idxp = idx_load(8);
    }
    __syncthreads();

    // Q: exterior-stem factors of column j (cells (k, j), k <= j - 4, two lane-sets):
    // INVMM(code) * ext(type, S[k-1], S[j+1]) -- static, gathered a step ahead
    float qf[2] = {0.f, 0.f};
    auto qfac = [&](int j) {
        if (j < 4 || j > N) return;
        const int sjp = (j < N) ? S[j + 1] : 5;
        const int sj = S[j];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int kk = 1 + h * WAVE + lane;
            const bool ok = kk <= j - 4;
            const int k = ok ? kk : 1;
            const int ix = off(j - k, N) + k - 1;
            const int ty = ptype(S[k], sj);
            const float e = L.dt[DT_EXT + ty * 36 + ((k > 1) ? S[k - 1] : 5) * 6 + sjp];
            qf[h] = ok ? ct[CT_INVMM + L.cc[ix]] * e : 0.f;
        }
    };
    if (wid == PX_WQ) qfac(4);
    const int s_end = N + 1;
    if (wid < PX_NB) {
#if PX_NB_CFG == 8
        // eight blocks (A/B, round 6): sizes 9, 14, 6, 13 of the four blocks the
        // stamps showed busiest (profiles/r06e_pf_cells_stamps.txt) on an eighth wave
        switch (wid) {
            case 0: pb_sweep<5, 22, 12, 11, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#if PX_PART != 5 && PX_PART < 8
            case 1: pb_sweep<4, 21, 19, 10, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
#if PX_PART != 7 && PX_PART < 8
            case 2: pb_sweep<3, 20, 18, 8, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
#if PX_PART == 1   // (A/B knobs) size 16 from block 4 to block 3
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 0, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 2   // size 16 from block 4 to block 5
            case 3: pb_sweep<28, 26, 1, 7, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 0, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 16, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 3   // size 0 from block 4 to block 3
            case 3: pb_sweep<28, 26, 1, 7, 0>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 16, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 5   // as 4, and size 0 from block 4 to block 1
            case 1: pb_sweep<4, 21, 19, 10, 0>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, -1, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 6   // size 16 from block 4 to block 5, size 15 from block 6 to block 3
            case 3: pb_sweep<28, 26, 1, 7, 15>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 0, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 16, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 7   // as 4, and size 13 from block 7 to block 2
            case 2: pb_sweep<3, 20, 18, 8, 13>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 0, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 8   // as 4, size 0 from block 4 to block 1 and size 13 from block 7 to block 2
            case 1: pb_sweep<4, 21, 19, 10, 0>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 2: pb_sweep<3, 20, 18, 8, 13>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, -1, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 9 || PX_PART == 10 || PX_PART == 11   // as 8, then 8 (9, 11) from block 2 and 15 (10, 11) from block 5 to block 4
            case 1: pb_sweep<4, 21, 19, 10, 0>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#if PX_PART == 10
            case 2: pb_sweep<3, 20, 18, 8, 13>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#else
            case 2: pb_sweep<3, 20, 18, 13, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#if PX_PART == 9
            case 4: pb_sweep<29, 27, 8, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 10
            case 4: pb_sweep<29, 27, 15, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#else
            case 4: pb_sweep<29, 27, 8, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#elif PX_PART == 4   // size 16 from block 4 to block 3, size 15 from block 6 to block 5
            case 3: pb_sweep<28, 26, 1, 7, 16>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 0, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#else
            case 3: pb_sweep<28, 26, 1, 7, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 16, 0, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 6: pb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
#if PX_PART == 7 || PX_PART >= 8
            default: pb_sweep<9, 14, 6, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#else
            default: pb_sweep<9, 14, 6, 13, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
#endif
        }
#else
        switch (wid) {
            // blocks of about equal LDS cost per lane-set (a size >= 6: 3 reads for
            // its special shapes + one per 4 generic ones; the small sizes ~3 per shape)
            // (round 5: 9, 13, 14 moved off the waves the stamps showed busiest,
            // profiles/r05w_pf_cells_stamps.txt: +0.7 %, profiles/r05_ab r05x)
            case 0: pb_sweep<5, 22, 12, 11, 9>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 1: pb_sweep<4, 21, 19, 10, 14>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 2: pb_sweep<3, 20, 18, 8, 6>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 3: pb_sweep<28, 26, 1, 7, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 4: pb_sweep<29, 27, 16, 0, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            case 5: pb_sweep<30, 2, 17, -1, -1>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
            default: pb_sweep<24, 25, 23, 15, 13>(L, XS, N, lane, wid, constrained, s_end PX_STP_ARGS); break;
        }
#endif
    } else {
        // the M / F / Q / R chains set the step time; issue arbitration favours the
        // older (B) waves of the workgroup, so these run at a higher priority
        __builtin_amdgcn_s_setprio(PX_ROLE_PRIO);
        // one sweep instance per role (round 6): each holds only its own role's
        // registers (the shared loop kept every role's values live: 38 SGPR spills)
        auto sweep = [&](auto role_c) __attribute__((always_inline)) {
        constexpr int ROLE = decltype(role_c)::value;   // 0 M, 1 F, 2 Q, 3 R
        for (int s = 4; s <= s_end; s++) {
            if constexpr (ROLE == 0) {
                // ---------------- M: qm items of span sq = s - 2, K lanes per item (a
                // power of two <= 16, one DPP row), split points in contiguous runs per
                // lane, summed over the K lanes:
                //   qm(i, jb)  = U(i, jb) + sum_{t >= 5} qm(i, i+t-1) qm1(i+t, jb)
                //   mla(i, sq) = the split part
                // with the unpaired part sum_t [t <= up_i] pw(t) qm1(i+t, jb) as the column
                // recursion U(i, jb) = qm1(i, jb) + [up_i >= 1] (expMLbase sigma) U(i+1, jb)
                // (split points t = 0..4 read no more: 894k -> 913k MC steps/s)
                // K follows the full fold's item count N - sq, so a refold sums every
                // item in the order a fold from scratch does (bit-identical tables)
                const int sq = s - 2;
                if (sq >= 4 && sq <= N - 3) {
                    const int lo = qlo(sq), n = qhi(sq) - lo + 1;
                    int K = 16;
                    while (K > 1 && (N - sq) * K > PX_NMW * WAVE) K >>= 1;
                    const int ipw = WAVE / K;                 // items per wave
                    const int mw = px_mw(wid);
                    const int k = lane & (K - 1);
                    const int item = mw * ipw + lane / K;
                    if (mw * ipw < n) {
                        const bool valid = item < n;
                        const int i = lo + (valid ? item : n - 1);
                        const int jb = i + sq, T = sq - 4;
                        // the split points t = 5..T only; the unpaired part is the
                        // column recursion U(i, jb) = qm1(i, jb) + [up_i >= 1] (expMLbase
                        // sigma) U(i+1, jb), U of span sq - 1 kept by the Q wave
                        // split points interleaved over the K lanes (lane k: t = 5 + k + K m),
                        // so an item's lanes read consecutive words of its qm1 column and qm
                        // row (no bank conflicts inside an item)
                        const int nit = T >= 5 ? (T - 4 + 2 * K - 1) / (2 * K) : 0;
                        const f2 *pq = L.q1 + colb(jb) + i - 1;   // qm1(i+t, jb) at +t
                        const f2 *pr = L.qm + rowb(i, N) - 5;      // qm(i, i+t-1) at +t (t >= 5)
                        const bool up1 = sq >= 5 && (!constrained || L.up[i] >= 1);
                        const f2 u1 = up1 ? L.uc[((sq - 1) & 1) * NP + jb] : f2{0.f, 0.f};
                        const f2 q0 = pq[0];
                        f2 A = {0.f, 0.f}, A1 = {0.f, 0.f};
                        const f2 z = {0.f, 0.f};
                        for (int m = 0; m < nit; m++) {   // t in A, t + K in A1 (past T: 0, whatever was read)
                            const int t = 5 + k + 2 * K * m, t2 = t + K;
                            const f2 qa = pq[t], qn = pq[t2], ra = pr[t], rn = pr[t2];
                            A = fma2(t <= T ? ra : z, t <= T ? qa : z, A);
                            A1 = fma2(t2 <= T ? rn : z, t2 <= T ? qn : z, A1);
                        }
                        A += A1;
                        if (K >= 2) A = dpp_add2<0xb1>(A);     // quad_perm [1,0,3,2]
                        if (K >= 4) A = dpp_add2<0x4e>(A);     // quad_perm [2,3,0,1]
                        if (K >= 8) A = dpp_add2<0x114>(A);    // row_shr:4
                        if (K >= 16) A = dpp_add2<0x118>(A);   // row_shr:8
                        if (valid && k == (K >= 8 ? K - 1 : 0)) {
                            L.qm[rowb(i, N) + sq - 4] = A + fma2(sp2(mlbase_sig), u1, q0);
                            L.mla[(sq & 1) * NP + i] = A;
                        }
                    }
                }
            } else if constexpr (ROLE == 1) {
                // ---------------- F: the changed cells of diagonal e = s - 1
                const int e = s - 1;
                if (e >= 4 && e <= N - 1) {
                    const int lo = clo(e), hi = chi(e);
                    for (int i0 = lo; i0 <= hi; i0 += WAVE) {
                        const int i = i0 + lane;
                        if (i > hi) break;
                        const int j = i + e;
                        const int ce = off(e, N) + i - 1, c1 = colb(j) + i - 1;
                        const f2 init = L.qb[ce];
                        const f2 stem = L.q1[c1];
                        const bool upj = e >= 5 && L.up[j] >= 1;
                        const f2 prev = upj ? L.q1[colb(j - 1) + i - 1] : f2{0.f, 0.f};
                        if (!is_mark2(init)) {
                            const int ty = ptype(S[i], S[j]);
                            const float mlcl = mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
                            f2 a_int = {0.f, 0.f};
                            if (e >= 6) {
                                const f2 *pp = L.part + ((e & 1) * 2 + ((i - 1) >> 6)) * PX_NB * WAVE + ((i - 1) & (WAVE - 1));
#pragma unroll
                                for (int b = 0; b < PX_NB; b++) a_int += pp[b * WAVE];
                            }
                            const f2 ml = e - 2 >= 4 ? L.mla[((e - 2) & 1) * NP + i + 1] : f2{0.f, 0.f};
                            const f2 qb = a_int + init + ml * sp2(mlcl);
                            const float mmc = L.dt[DT_MMI + L.cc[ce]];
                            L.qb[ce] = qb * sp2(mmc) + f2{0.f, 0.f};   // never the mark (-0)
                            L.q1[c1] = fma2(qb, stem, prev * sp2(mlbase_sig));
                        } else {
                            L.q1[c1] = prev * sp2(mlbase_sig);
                        }
                    }
                }
            } else if constexpr (ROLE == 2) {
                // ---------------- Q: q5[j], j = s - 1 (column j is final); the
                // exterior factors of column j + 1 are gathered one step ahead
                const int j = s - 1;
                if (j >= 4 && j <= N && (!incr || j >= m_lo - 1)) {
                    f2 acc = {0.f, 0.f};
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        if (h * WAVE >= j - 4) break;
                        const int kk = 1 + h * WAVE + lane;
                        const int k = kk <= j - 4 ? kk : 1;
                        const int ix = off(j - k, N) + k - 1;
                        acc = fma2(L.q5[k - 1] * L.qb[ix], sp2(qf[h]), acc);
                    }
                    acc = wave_sum_f2(acc);
                    if (lane == 0) L.q5[j] = (L.up[j] >= 1 ? L.q5[j - 1] * sp2(sig1) : f2{0.f, 0.f}) + acc;
                }
                {   // U(i, jb) of span sq = s - 2 for every cell (M reads it next step)
                    const int sq = s - 2;
                    if (sq >= 4 && sq <= N - 4) {
                        for (int i = 1 + lane; i <= N - sq; i += WAVE) {
                            const int jb = i + sq;
                            const bool up1 = sq >= 5 && (!constrained || L.up[i] >= 1);
                            const f2 u1 = up1 ? L.uc[((sq - 1) & 1) * NP + jb] : f2{0.f, 0.f};
                            L.uc[(sq & 1) * NP + jb] = fma2(sp2(mlbase_sig), u1, L.q1[colb(jb) + i - 1]);
                        }
                    }
                }
                qfac(j + 1);
            } else {
                // ---------------- R: records of diagonal s + 2 (B loads them next step for
                // the step after), tables of s + 3, bases of s + 4, rank list of s + 5
                rec_store(s + 2, pend);
                pend = rec_load(s + 3, seqp);
                seqp = seq_load(s + 4, idxp);
                idxp = idx_load(s + 5);
            }
            PSTAMP(4);
            lds_barrier();
            PSTAMP(6);
        }
        };
        if (px_mw(wid) >= 0) sweep(std::integral_constant<int, 0>{});
        else if (wid == PX_WF) sweep(std::integral_constant<int, 1>{});
        else if (wid == PX_WQ) sweep(std::integral_constant<int, 2>{});
        else sweep(std::integral_constant<int, 3>{});   // PX_WR
    }
#ifdef ADX_STAMP
    if (lane == 0)
        for (int k = 0; k < 12; k++) atomicAdd(&g_stamps_p[wid][k], st_acc[k]);
#endif
    __syncthreads();
    // ---- the proposal's tables (the next step's unchanged cells) and the energies
    if (dst) {
        for (int k = tid; k < C; k += PX_NT) {
            const f2 a = L.qb[k], b = L.qm[k], c = L.q1[k];
            dst[k] = a.x;
            dst[B1 + k] = a.y;
            dst[Cs + k] = b.x;
            dst[B1 + Cs + k] = b.y;
            dst[2 * Cs + k] = c.x;
            dst[B1 + 2 * Cs + k] = c.y;
        }
        for (int k = tid; k <= N; k += PX_NT) {
            dst[3 * Cs + k] = L.q5[k].x;
            dst[B1 + 3 * Cs + k] = L.q5[k].y;
        }
        for (int k = tid; k < ((C + 15) >> 4); k += PX_NT) cc_dst[k] = reinterpret_cast<const uint4 *>(L.cc)[k];
    }
    if (tid == 0) {   // ensemble energy -kT (ln Z_scaled - N ln sigma), as vrna_pf (float)
        const f2 z = L.q5[N];
        gout[size_t(w) * ka.n_variants + vs0] = float(-XS->kT * (log(double(z.x)) - N * XS->log_sigma));
        gout[size_t(w) * ka.n_variants + vs1] = float(-XS->kT * (log(double(z.y)) - N * XS->log_sigma));
    }
}

}  // namespace

// LDS bytes of the lanes = cells PF kernel for this workload (0: not covered)
size_t pf_cells_lds(const KArgs &ka) {
    if (ka.mode != 0 || ka.Nmax > PX_NMAX || ka.Nmax < 8) return 0;
    const size_t b = PxLay(ka.Nmax).BYTES;   // no static LDS (block_or, not __syncthreads_or)
    return b <= 160 * 1024 ? b : 0;
}

hipError_t launch_pf_cells(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, float *gout,
                           hipStream_t stream) {
    const size_t lds = pf_cells_lds(ka);
    if (lds == 0) return hipErrorInvalidValue;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(pf_cells_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(pf_cells_kernel, dim3(W * ka.n_groups2), dim3(PX_NT), lds, stream, ka, ka.X, seqs, W, mask,
                       gout);
    return hipGetLastError();
}

}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_pf(unsigned long long *out, int reset) {  // [16][12]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_p), sizeof(adx::g_stamps_p)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][12] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_p), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
