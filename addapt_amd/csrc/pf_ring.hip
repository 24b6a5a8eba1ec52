// gfx950 McCaskill inside pass for folds longer than pf_cells.hip covers
// (BASELINE config 4: N = 150, the reference's vrna_pf at scoring.cc:58,65),
// lanes = cells like pf_cells_kernel, with the LDS carved for ONE fold:
//
//   * one workgroup (14 waves) per (walker, variant): FP32 values (pf_cells
//     keeps apo|holo as float2, which at N = 150 would need 257 KB);
//   * qm (row-major) and qm1 (column-major) stay whole in LDS (2 x 43 KB);
//   * qb and the inner codes live in a RING of the last 34 diagonals: an
//     interior loop (<= 30 unpaired) reaches 32 diagonals back, F writes the
//     previous one and the prep stage the next;
//   * the exterior recursion q5[j] needs whole columns of qb: F stores every
//     finalised cell to the walker's table slot (diagonal-major, as pf_cells),
//     the prep stage stores the restored and non-pairable cells, and Q reads
//     column j from there two steps after it is final (a global read per lane
//     and lane-set, issued a step ahead; every writer drains its stores at the
//     start of its next step, so no wave waits on a store on its way to the
//     barrier);
//   * the slot keeps qm and qm1 DIAGONAL-major (not row- / column-major as
//     pf_cells): the outside pass for these lengths (outside_ring.hip) reads
//     them from the slot with lanes = cells, where a diagonal-major table makes
//     every read one coalesced line.
//
// One step = one anti-diagonal, ONE barrier:
//   B  (waves 0-6)  interior-loop sums of diagonal s (pf_cells' blocks)
//   F  (wave 7)     cells of diagonal s-1: qb, qm1, the slot store
//   Q  (wave 8)     q5[s-3] from column s-3 (loaded last step), the load of
//                   column s-2
//   R  (wave 9)     setup records of the B lanes, four stages a step apart
//   prep            of diagonal s+1, one lane-set each on M waves 12, 13 and R: inner
//                   codes, hairpin (+ motif) initial values of the changed
//                   cells, restored values of the others (loaded a step ahead)
//   M  (waves 10-13) qm items of span s-2
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {
namespace {

constexpr int RG_NW = 14;
#ifndef RG_PART
#define RG_PART 0   // interior-loop size partition of the seven blocks (A/B knob)
#endif
constexpr int RG_NT = RG_NW * WAVE;
constexpr int RG_NB = 7;              // interior-loop blocks (waves 0..6)
constexpr int RG_NMW = 4;             // qm item waves
constexpr int RG_WF = 7, RG_WQ = 8, RG_WR = 9;
__host__ __device__ constexpr int rg_mw(int w) {   // M wave index (0 = most items) or -1
    return w == 10 ? 0 : w == 11 ? 1 : w == 13 ? 2 : w == 12 ? 3 : -1;
}
constexpr int RG_NMIN = 101;          // pf_cells_kernel covers N <= 100
constexpr int RG_NMAX = 190;          // lane-sets of a diagonal: N - 4 <= RG_SETS * 64
constexpr int RG_SETS = 3;
constexpr int RG_RING = 34;           // diagonals s-32 .. s+1
constexpr int RG_RF = 8;              // record fields: word, mmo, mo, m23, 1x1..2x2 factors
constexpr int RG_SLACK = 16;

struct RgLay {
    int C, NP, RS;
    size_t QM, Q1, QB, CC, PART, REC, CL, MLA, UC, Q5, CT, DT, PW, BY, MT, BYTES;
    __host__ __device__ static size_t a16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ explicit RgLay(int N) {
        C = ((N - 4) * (N - 3)) / 2;
        NP = N + 2;
        RS = ((N - 4) + 3) & ~3;                                   // ring row: the longest diagonal
        size_t o = 0;
        QM = o;   o += a16((size_t(C) + RG_SLACK) * 4);           // qm, row-major
        Q1 = o;   o += a16((size_t(C) + RG_SLACK) * 4);           // qm1, column-major
        QB = o;   o += a16(size_t(RG_RING) * RS * 4);             // qb * mismatchI(inner) ring
        CC = o;   o += a16(size_t(RG_RING) * RS);                 // inner-pair code ring
        PART = o; o += a16(size_t(2) * RG_SETS * RG_NB * WAVE * 4);   // [parity][lane-set][block][lane]
        REC = o;  o += a16(size_t(2) * RG_SETS * RG_RF * WAVE * 4 + 16);   // [parity][set][field][lane]; counts
        CL = o;   o += a16(size_t(C) + size_t(NP));               // rank lists of the changed pairable cells + counts
        MLA = o;  o += a16(size_t(2) * NP * 4);                   // split part of qm, by span parity
        UC = o;   o += a16(size_t(2) * NP * 4);                   // unpaired part U(i, j) of qm by column j, by span parity
        Q5 = o;   o += a16(size_t(NP) * 4);
        CT = o;   o += a16(size_t(CT_SIZE) * 4);
        DT = o;   o += a16(size_t(DT_HP + N + 1) * 4);
        PW = o;   o += a16(size_t(N + 9) * 4);                    // (expMLbase sigma)^t
        BY = o;   o += a16(size_t(7) * NP);                       // S, up, dn, ptn, enc, flg, mat
        MT = o;   o += a16(size_t(MAX_SPECIAL_HP) * 8 + 2 * MAX_MOTIF);
        BYTES = o;
    }
};

struct RgL {
    float *qm, *q1, *qb, *part, *mla, *uc, *q5, *rec, *ct, *dt, *pw;
    int *rcnt;
    uint8_t *cc, *cl, *cn, *S, *up, *dn, *ptn, *enc, *flg, *mat;
    int N, NP, RS;
};

// ring position of diagonal D's first cell
__device__ __forceinline__ int rgo(int D, int RS) { return (D % RG_RING) * RS; }

__device__ __forceinline__ bool rg_allowed(const RgL &L, int i, int j) {   // kernels.hip allowed()
    const int fi = L.flg[i], fj = L.flg[j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[i], pj = L.ptn[j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[i] == L.enc[j];
}

__host__ __device__ constexpr int rkind(int n1, int n2) {
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
__device__ __forceinline__ float rshape_factor(const DevScaled *XS, int u, int n1) {
    const int kd = rkind(n1, u - n1);
    return kd < 0 ? XS->fgen[(u - 6) * FG_ROW + n1 - 2]
         : kd == TK_STK ? XS->ctab[CT_FSM + 0]
         : kd == TK_B1 ? XS->ctab[CT_FSM + 1]
         : kd == TK_BUL ? XS->ctab[CT_FB + u]
         : kd == TK_1N ? XS->ctab[CT_F1N + u - 1]
         : kd == TK_I11 ? XS->ctab[CT_FSM + 2]
         : kd == TK_I22 ? XS->ctab[CT_FSM + 4]
         : kd == TK_M23 ? XS->ctab[CT_FSM + 5]
         : XS->ctab[CT_FSM + 3];
}

struct RgCell {              // per lane: the closing pair (i, i+s)
    int i, ty8, A, B;
    float tau, mo, m23;
    float t11, t12, t21, t22;
};

// One shape (N1, U - N1) of a size <= 5: the inner cell at qb / cc + N1 (this
// lane's ring bases on diagonal s-2-U).
template <int U, int N1, bool MK>
__device__ __forceinline__ void rshape1(const RgL &L, const RgCell &c, const float *fv, const float *qb,
                                        const uint8_t *cc, uint32_t bits, float &g, float &sp) {
    constexpr int k = rkind(N1, U - N1);
    constexpr int FI = N1 < U - N1 ? N1 : U - N1;
    float v = qb[N1];
    if constexpr (MK) v *= float((bits >> N1) & 1u);
    if constexpr (k < 0) {
        g = fmaf(v, fv[FI], g);
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
        sp = fmaf(v, f, sp);
    }
}
template <int U, bool MK, int... N1s>
__device__ __forceinline__ void rshape_seq(std::integer_sequence<int, N1s...>, const RgL &L, const RgCell &c,
                                           const float *fv, const float *qb, const uint8_t *cc, uint32_t bits,
                                           float &g, float &sp) {
    (rshape1<U, N1s, MK>(L, c, fv, qb, cc, bits, g, sp), ...);
}
template <int U>
struct RgSize {
    float fv[U < 0 ? 1 : U / 2 + 1];
    __device__ __forceinline__ void load(const DevScaled *XS) {
        if constexpr (U >= 0)
#pragma unroll
            for (int n1 = 0; n1 <= U / 2; n1++) fv[n1] = rshape_factor(XS, U, n1);
    }
    template <bool MK>
    __device__ __forceinline__ void run(const RgL &L, const RgCell &c, int s, int umax, float &g, float &sp) const {
        if constexpr (U >= 0) {
            if (U <= umax) {
                const int o = rgo(s - 2 - U, L.RS) + c.i;   // inner cell (i+1+n1, ...) at o + n1
                uint32_t bits = 0;
                if constexpr (MK) {
                    const int lo = max(0, U - c.B), hi = min(U, c.A);
                    bits = hi < lo ? 0u : ((2u << hi) - 1u) & ~((1u << lo) - 1u);
                }
                rshape_seq<U, MK>(std::make_integer_sequence<int, U + 1>{}, L, c, fv, L.qb + o, L.cc + o, bits, g, sp);
            }
        }
    }
};
// Loop size U >= 6 over the four lanes of a cell (pf_cells.hip PxSizeQ)
template <int U>
struct RgSizeQ {
    static constexpr int NR = U >= 6 ? (U - 3 + 3) / 4 : 1;
    float gf[NR];
    float fsp;
    int n1sp;
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
    __device__ __forceinline__ void run(const RgL &L, const RgCell &c, int s, int umax, int r, int ctb, float outer,
                                        float &g, float &sp) const {
        if (U <= umax) {
            const int o = rgo(s - 2 - U, L.RS) + c.i;
            uint32_t bits = ~0u;
            if constexpr (MK) {
                const int lo = max(0, U - c.B), hi = min(U, c.A);
                bits = hi < lo ? 0u : ((2u << hi) - 1u) & ~((1u << lo) - 1u);
            }
            {
                float v = L.qb[o + n1sp];
                if constexpr (MK) v *= float((bits >> n1sp) & 1u);
                const int ci = L.cc[o + n1sp];
                sp = fmaf(v, L.ct[ctb + ci] * (outer * fsp), sp);
            }
            const float *q = L.qb + o + 2 + r;
            const uint32_t bm = bits >> (2 + r);
#pragma unroll
            for (int m = 0; m < NR; m++) {
                float v = q[4 * m];
                if constexpr (MK) v *= float((bm >> (4 * m)) & 1u);
                g = fmaf(v, gf[m], g);
            }
        }
    }
};
template <int U>
struct RgBlk {
    using T = typename std::conditional<(U < 0), RgSize<-1>, typename std::conditional<(U <= 5), RgSize<U>, RgSizeQ<U>>::type>::type;
};
#ifndef ADX_SMALL_R0
#define ADX_SMALL_R0 1   // sizes <= 5 on phase 0 only (the other phases' copies are discarded)
#endif
template <int U, bool MK>
__device__ __forceinline__ void rg_run(const typename RgBlk<U>::T &z, const RgL &L, const RgCell &c, int s, int umax,
                                       int r, int ctb, float outer, float &g, float &sp, float &gs, float &sps) {
    if constexpr (U < 0) {
    } else if constexpr (U <= 5) {
        if (!ADX_SMALL_R0 || r == 0) z.template run<MK>(L, c, s, umax, gs, sps);   // counted on phase 0 only
    } else {
        z.template run<MK>(L, c, s, umax, r, ctb, outer, g, sp);
    }
}
template <int U>
__device__ __forceinline__ void rg_load(typename RgBlk<U>::T &z, const DevScaled *XS, int r) {
    if constexpr (U < 0) {
    } else if constexpr (U <= 5) {
        z.load(XS);
    } else {
        z.load(XS, r);
    }
}
__device__ __forceinline__ float quad_sum_r(float v) {   // sum over the 4 lanes of a quad, in every lane
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));   // [1,0,3,2]
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));   // [2,3,0,1]
}
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the wave, uniform result: DPP row sums, then the four rows' totals
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v = dpp_add<0xb1>(v);    // quad_perm [1,0,3,2]
    v = dpp_add<0x4e>(v);    // quad_perm [2,3,0,1]
    v = dpp_add<0x114>(v);   // row_shr:4
    v = dpp_add<0x118>(v);   // row_shr:8 -> lane 15 of each row holds the row sum
    const int b = __float_as_int(v);
    return __int_as_float(__builtin_amdgcn_readlane(b, 15)) + __int_as_float(__builtin_amdgcn_readlane(b, 31)) +
           __int_as_float(__builtin_amdgcn_readlane(b, 47)) + __int_as_float(__builtin_amdgcn_readlane(b, 63));
}
#ifdef ADX_STAMP
// Diagnostic build only: per-wave cycle sums of the phases (s_memtime), read
// back through adx_debug_stamps_ring().  Never in the product.
__device__ unsigned long long g_stamps_r[16][8];
#define RSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#define RG_STP_PARAMS , unsigned long long *st_acc, unsigned long long &st_last
#define RG_STP_ARGS , st_acc, st_last
#else
#define RSTAMP(k) do { } while (0)
#define RG_STP_PARAMS
#define RG_STP_ARGS
#endif

// global stores of this wave complete before the step's barrier (the slot is
// read back by Q within the workgroup)
__device__ __forceinline__ void vm_drain() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// B: interior-loop sums of every diagonal for one block of loop sizes (pf_cells.hip pb_sweep)
template <int U0, int U1, int U2, int U3, int U4>
__device__ __forceinline__ void rb_sweep(const RgL &L, const DevScaled *XS, int N, int lane, int wid,
                                         bool constrained, int s_end RG_STP_PARAMS) {
    constexpr auto tb = [](int u) { return u >= 2 && u <= 4; };
    constexpr bool TB = tb(U0) || tb(U1) || tb(U2) || tb(U3) || tb(U4);
    constexpr bool H5 = U0 == 5 || U1 == 5 || U2 == 5 || U3 == 5 || U4 == 5;
    const float eTAU = XS->ctab[CT_FSM + 6];
    const int r = lane & 3, cq = lane >> 2;
    typename RgBlk<U0>::T s0;
    typename RgBlk<U1>::T s1;
    typename RgBlk<U2>::T s2;
    typename RgBlk<U3>::T s3;
    typename RgBlk<U4>::T s4;
    rg_load<U0>(s0, XS, r);
    rg_load<U1>(s1, XS, r);
    rg_load<U2>(s2, XS, r);
    rg_load<U3>(s3, XS, r);
    rg_load<U4>(s4, XS, r);
    const int ctb = r < 2 ? CT_BUL : CT_ONEN;
    for (int s = 4; s <= s_end; s++) {
        const int par = s & 1;
        const int umax = min(30, s - 6);
        const int ncell = (s <= N - 1 && umax >= 0) ? uni(L.rcnt[par]) : 0;
        for (int c0 = 0; c0 < ncell; c0 += WAVE / 4) {
            const int idx = c0 + cq;
            const float *rr = L.rec + ((par * RG_SETS + (idx >> 6)) * RG_RF) * WAVE + (idx & (WAVE - 1));
            // word: i | ty << 8 | A << 11 | B << 19 | masked << 27 | real << 28
            const int fl = __float_as_int(rr[0]);
            RgCell c;
            c.i = fl & 255;
            const int ty = (fl >> 8) & 7;
            c.ty8 = ty * 8;
            c.A = (fl >> 11) & 255;
            c.B = (fl >> 19) & 255;
            const float mmo = rr[WAVE];
            c.tau = ty > 2 ? eTAU : 1.f;
            c.mo = rr[2 * WAVE];
            c.m23 = H5 ? rr[3 * WAVE] : 0.f;
            c.t11 = c.t12 = c.t21 = c.t22 = 0.f;
            if constexpr (TB) {
                c.t11 = rr[4 * WAVE];
                c.t12 = rr[5 * WAVE];
                c.t21 = rr[6 * WAVE];
                c.t22 = rr[7 * WAVE];
            }
            const float outer = r < 2 ? c.tau : c.mo;
            float g = 0.f, sp = 0.f, gs = 0.f, sps = 0.f;
            RSTAMP(1);   // B cell records
            const bool mk = constrained && __ballot((fl >> 27) & 1) != 0;
            if (mk) {
                rg_run<U0, true>(s0, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U1, true>(s1, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U2, true>(s2, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U3, true>(s3, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U4, true>(s4, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
            } else {
                rg_run<U0, false>(s0, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U1, false>(s1, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U2, false>(s2, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U3, false>(s3, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
                rg_run<U4, false>(s4, L, c, s, umax, r, ctb, outer, g, sp, gs, sps);
            }
            const float part = quad_sum_r(fmaf(g, mmo, sp) + (r == 0 ? fmaf(gs, mmo, sps) : 0.f));
            if (r == 0 && idx < ncell && ((fl >> 28) & 1))
                L.part[((par * RG_SETS + ((c.i - 1) >> 6)) * RG_NB + wid) * WAVE + ((c.i - 1) & (WAVE - 1))] = part;
            RSTAMP(2);   // B shapes
        }
        RSTAMP(3);
        lds_barrier();
        RSTAMP(7);   // barrier
    }
}

// One workgroup per (walker, variant of a groups2 pair).  gout: [W][n_variants]
// ensemble energies (kcal/mol); qscr: per workgroup C floats of qb when the fold
// keeps no state (adx_score_batch), else null (the slot holds qb).
__global__ void __launch_bounds__(RG_NT, 1)
pf_ring_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, const int *mask,
               float *gout, float *qscr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ng = 2 * ka.n_groups2;
    const int wb = blockIdx.x / ng, rem = blockIdx.x % ng;
    const int grp = rem >> 1, half = rem & 1;
    if (wb >= W) return;
    const WalkerRef wr = walker_ref(ka, mask, wb);   // heaviest refolds first
    if (!wr.on) return;
    const int w = wr.w;
    const int v0 = ka.groups2[2 * grp], vh = ka.groups2[2 * grp + half];
    if (half == 1 && vh == v0) return;   // a lone variant: one fold
    const DevVariant V = ka.variants[vh];
    const bool hol = V.motif != 0;
    const int N = uni(V.N);
    const RgLay Y(N);
    RgL L;
    L.qm = reinterpret_cast<float *>(smem + Y.QM);
    L.q1 = reinterpret_cast<float *>(smem + Y.Q1);
    L.qb = reinterpret_cast<float *>(smem + Y.QB);
    L.cc = reinterpret_cast<uint8_t *>(smem + Y.CC);
    L.part = reinterpret_cast<float *>(smem + Y.PART);
    L.rec = reinterpret_cast<float *>(smem + Y.REC);
    L.rcnt = reinterpret_cast<int *>(smem + Y.REC + size_t(2) * RG_SETS * RG_RF * WAVE * 4);
    L.cl = reinterpret_cast<uint8_t *>(smem + Y.CL);
    L.cn = L.cl + Y.C;
    L.mla = reinterpret_cast<float *>(smem + Y.MLA);
    L.uc = reinterpret_cast<float *>(smem + Y.UC);
    L.q5 = reinterpret_cast<float *>(smem + Y.Q5);
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
    uint32_t *spk = reinterpret_cast<uint32_t *>(smem + Y.MT);
    float *spv = reinterpret_cast<float *>(smem + Y.MT + MAX_SPECIAL_HP * 4);
    uint8_t *mcode = reinterpret_cast<uint8_t *>(smem + Y.MT + MAX_SPECIAL_HP * 8);
    int8_t *mpt = reinterpret_cast<int8_t *>(mcode + MAX_MOTIF);
    L.N = N;
    L.NP = Y.NP;
    L.RS = Y.RS;
    // RG_WPERM (diagnostic builds): physical wave -> role, to try other role / SIMD pairings
#ifdef RG_WPERM
    constexpr int wperm[RG_NW] = {RG_WPERM};
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(wperm[tid / WAVE]);
#else
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
#endif
    const int C = Y.C, NP = Y.NP, RS = Y.RS;
    const DevTables &T = *ka.T;
#ifdef ADX_STAMP
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

    // ---- incremental fold state (pf_cells.hip): this variant's tables of the
    // current sequence (src) and the proposal's (dst), diagonal-major
    const size_t Cs = size_t(ka.cells), B1 = 3 * Cs + size_t(ka.Nmax) + 2;
    const float *src = nullptr;
    float *dst = nullptr;
    int m_lo = 0, m_hi = 0;
    if (ka.tab) {
        const int cur = wr.cur;
        float *base = ka.tab + size_t(w) * 2 * ka.tab_slot;
        dst = base + size_t(1 - cur) * ka.tab_slot + size_t(grp) * 2 * B1 + size_t(half) * B1;
        if (wr.valid && wr.c0 >= 0) {
            src = base + size_t(cur) * ka.tab_slot + size_t(grp) * 2 * B1 + size_t(half) * B1;
            m_lo = wr.c0 + 1 + V.before_len;
            m_hi = wr.c1 + 1 + V.before_len;
        }
    }
    // qb of every cell, read back by Q: the slot, or this workgroup's scratch
    float *qbg = dst ? dst : qscr + size_t(blockIdx.x) * Cs;
    const bool incr = src != nullptr;
    m_lo = uni(m_lo);
    m_hi = uni(m_hi);
    auto clo = [&](int D) { return incr ? max(1, m_lo - 1 - D) : 1; };
    auto chi = [&](int D) { return incr ? min(N - D, m_hi + 1) : N - D; };
    auto qlo = [&](int sq) { return incr ? max(1, m_lo - 2 - sq) : 1; };
    auto qhi = [&](int sq) { return incr ? min(N - sq, m_hi + 2) : N - sq; };

    // ---- sequence, constraint arrays, tables (round 6, as pf_cells.hip): the one or
    // two elements of each this thread stores, all loads in flight at once, then the
    // stores (a loop per table waited on each load in turn)
    static_assert(288 <= RG_NT && RG_NMAX + 9 <= RG_NT && MAX_SPECIAL_HP <= RG_NT && MAX_MOTIF <= RG_NT,
                  "one setup element per thread");
    constexpr int NCT = (CT_SIZE + RG_NT - 1) / RG_NT;
    float v_ct[NCT];
#pragma unroll
    for (int t = 0; t < NCT; t++) v_ct[t] = XS->ctab[min(tid + t * RG_NT, CT_SIZE - 1)];
    const float v_mh = (&T.mmH[0][0][0])[min(tid, 199)], v_mi = (&T.mmI[0][0][0])[min(tid, 199)],
                v_ms = (&T.mlstem[0][0][0])[min(tid, 199)];
    const float v_ex = (&T.ext[0][0][0])[min(tid, 287)], v_tau = T.termAU[tid & 7];
    const float v_hp = XS->hp[min(tid, N)], v_pw = XS->pwml[min(tid, N + 8)];
    const int n_sp = XS->n_special;
    const uint32_t v_spk = XS->sp_key[min(tid, MAX_SPECIAL_HP - 1)];
    const float v_spv = XS->sp_val[min(tid, MAX_SPECIAL_HP - 1)];
    const uint8_t v_mc = XS->motif_code[min(tid, MAX_MOTIF - 1)];
    const int8_t v_mp = XS->motif_pt[min(tid, MAX_MOTIF - 1)];
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
    static_assert(RG_NMAX + 2 <= RG_NT, "one position per thread");
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
#pragma unroll
    for (int t = 0; t < NCT; t++)
        if (tid + t * RG_NT < CT_SIZE) L.ct[tid + t * RG_NT] = v_ct[t];
    if (tid < 200) {
        L.dt[DT_MMH + tid] = v_mh;
        L.dt[DT_MMI + tid] = v_mi;
        L.dt[DT_MLS + tid] = v_ms;
    }
    if (tid < 288) L.dt[DT_EXT + tid] = v_ex;
    if (tid < 8) L.dt[DT_TAU + tid] = v_tau;
    if (tid <= N) L.dt[DT_HP + tid] = v_hp;
    if (tid < N + 9) L.pw[tid] = v_pw;
    if (tid < MAX_SPECIAL_HP) {
        const bool on = tid < n_sp;
        spk[tid] = on ? v_spk : 0xFFFFFFFFu;
        spv[tid] = on ? v_spv : 0.f;
    }
    if (tid < MAX_MOTIF) {
        mcode[tid] = v_mc;
        mpt[tid] = v_mp;
    }
    for (int k = tid; k < 2 * NP; k += RG_NT) L.mla[k] = 0.f;
    for (int k = C + tid; k < C + RG_SLACK; k += RG_NT) L.qm[k] = L.q1[k] = 0.f;
    for (int k = tid; k < RG_RING * RS; k += RG_NT) {
        L.qb[k] = 0.f;
        L.cc[k] = 0;
    }
    const bool constrained = __syncthreads_or(cst);
    if (tid == 0) {   // ViennaRNA's S1 wrap-around
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
    }
    const int mL = XS->motif_len;
    const bool any_motif = hol && mL > 0;
    __syncthreads();
    if (any_motif) {
        for (int o = tid + 1; o + mL - 1 <= N; o += RG_NT) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) ok = L.S[o + k] == mcode[k];
            L.mat[o] = ok ? 1 : 0;
        }
        __syncthreads();
        for (int o = 1 + wid; o + mL - 1 <= N; o += RG_NW) {
            if (!uni(L.mat[o])) continue;
            bool ok = true;
            for (int k = lane; k < mL; k += WAVE) {
                const int pk = mpt[k];
                if (pk < 0) ok = ok && L.up[o + k] >= 1;
                else if (pk > k) ok = ok && rg_allowed(L, o + k, o + pk);
            }
            const bool all = __ballot(!ok) == 0;
            if (lane == 0) L.mat[o] = all ? 1 : 0;
        }
    }
    // ---- refold restore of qm (row-major) and qm1 (column-major) from the
    // slot's diagonal-major tables, one diagonal per wave, lanes = cells; a fold
    // from scratch zeroes qm (spans N-2, N-1 are never computed)
    if (incr) {
        // this wave's (diagonal, lane-set) items in batches of RB: every load of a
        // batch in flight before its stores (round 6; a load -> store pair per item
        // waited on HBM once per item)
        constexpr int RB = 8;
        int D = 4 + wid, i0 = 1;
        const float q5v = src[3 * Cs + min(tid, N)];
        while (D <= N - 1) {
            float va[RB], vb[RB];
            int ia[RB], ib[RB];
#pragma unroll
            for (int k = 0; k < RB; k++) {
                const int i = i0 + lane;
                const bool ok = D <= N - 1 && i <= N - D;
                const int c = ok ? off(D, N) + i - 1 : 0;
                va[k] = src[Cs + c];
                vb[k] = src[2 * Cs + c];
                ia[k] = ok ? rowb(i, N) + D - 4 : -1;
                ib[k] = colb(i + D) + i - 1;
                if (D <= N - 1) {   // next item (uniform)
                    i0 += WAVE;
                    if (i0 > N - D) {
                        D += RG_NW;
                        i0 = 1;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < RB; k++)
                if (ia[k] >= 0) {
                    L.qm[ia[k]] = va[k];
                    L.q1[ib[k]] = vb[k];
                }
        }
        if (tid <= m_lo - 2 && tid <= N) L.q5[tid] = q5v;
    } else {
        for (int k = tid; k < C; k += RG_NT) L.qm[k] = 0.f;
    }
    __syncthreads();
    const uint8_t *S = L.S;
    const float *ct = L.ct;
    const float sig1 = XS->sig[1], mlbase_sig = XS->mlbase_sig, mlclosing = XS->mlclosing;
    const float mext = XS->motif_extra;
    const int nsp = XS->n_special < MAX_SPECIAL_HP ? XS->n_special : MAX_SPECIAL_HP;

    // the changed cells' multiloop stems in qm1 (F reads them before it
    // overwrites them) and the rank lists of the changed pairable cells (the B
    // lanes): cl[off(D) + rank] = i, cn[D] = count
    for (int D = 4 + wid; D <= N - 1; D += RG_NW) {
        const int od = off(D, N), lo = clo(D), hi = chi(D);
        int base = 0;
        for (int i0 = lo; i0 <= hi; i0 += WAVE) {   // the changed band's rows (round 6: every row before)
            const int i = i0 + lane;
            const bool inb = i <= hi;
            bool pr = false;
            if (inb) {
                const int j = i + D;
                const int type = ptype(S[i], S[j]);
                pr = type != 0 && rg_allowed(L, i, j);
                L.q1[colb(j) + i - 1] = pr ? L.dt[DT_MLS + type * 25 + S[i - 1] * 5 + S[j + 1]] : 0.f;
            }
            const uint64_t m = __ballot(pr);
            const int slot = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
            if (pr) L.cl[od + slot] = uint8_t(i);
            base += __popcll(m);
        }
        if (lane == 0) L.cn[D] = uint8_t(base);
    }
    for (int k = tid; k <= 3 && k <= N; k += RG_NT) {   // q5[0..3]: unpaired prefix
        float q = 1.f;
        bool ok = true;
        for (int t = 1; t <= k; t++) {
            ok = ok && L.up[t] >= 1;
            q *= sig1;
        }
        L.q5[k] = ok ? q : 0.f;
    }
    __syncthreads();

    // ---- prep of lane-set h of diagonal D into the ring (lane-sets 0, 1, 2 on
    // waves 12, 13 and R): inner codes; the changed cells' hairpin (+ motif)
    // initial values or the non-pairable mark (-0, also stored to the slot); the
    // restored values of the others (loaded one step ahead: rload) and their
    // slot copies
    float rsv = 0.f;
    auto rload = [&](int D, int h) {
        if (!incr || D < 4 || D > N - 1) return;
        const int od = off(D, N), lo = clo(D), hi = chi(D);
        const int i = 1 + h * WAVE + lane;
        if (h * WAVE < N - D && i <= N - D && (i < lo || i > hi)) rsv = src[od + i - 1];
    };
    auto prep = [&](int D, int h) {
        if (D < 4 || D > N - 1) return;
        const int od = off(D, N), ro = rgo(D, RS), lo = clo(D), hi = chi(D);
        {
            const int i = 1 + h * WAVE + lane;
            if (h * WAVE >= N - D || i > N - D) return;
            const int j = i + D;
            const int type = ptype(S[i], S[j]);
            L.cc[ro + i - 1] = uint8_t(rtype(type) * 25 + S[j + 1] * 5 + S[i - 1]);
            if (i >= lo && i <= hi) {
                const bool pr = type != 0 && rg_allowed(L, i, j);
                float init = -0.f;
                if (pr) {
                    const int u = D - 1;
                    float h0 = 0.f;
                    if (L.up[i + 1] >= u) {
                        bool special = false;
                        if (u == 3 || u == 4 || u == 6) {
                            const int sh = special_hp(spk, hp_key(S, i, u + 2));
                            if (sh >= 0) {
                                h0 = spv[sh];
                                special = true;
                            }
                        }
                        if (!special)
                            h0 = L.dt[DT_HP + u] * ((u == 3) ? L.dt[DT_TAU + type]
                                                             : L.dt[DT_MMH + type * 25 + S[i + 1] * 5 + S[j - 1]]);
                    }
                    const bool mx = hol && D == mL - 1 && mL > 0 && L.mat[i];
                    init = mx ? h0 + mext : h0;
                } else {
                    qbg[od + i - 1] = -0.f;   // non-pairable: the mark, final
                }
                L.qb[ro + i - 1] = init;
            } else {   // restored (final)
                L.qb[ro + i - 1] = rsv;
                qbg[od + i - 1] = rsv;
            }
        }
    };
    // this wave's prep lane-set: the two M waves with the fewest items and R
    const int ph = wid == 12 ? 0 : wid == 13 ? 1 : wid == RG_WR ? 2 : -1;

    // ---- records (wave R): pf_cells.hip's four stages, three lane-sets
    struct Pend {
        int n;
        int w1[RG_SETS];
        float mmo[RG_SETS], mo[RG_SETS], m23[RG_SETS], t11[RG_SETS], t12[RG_SETS], t21[RG_SETS], t22[RG_SETS];
    };
    struct Seq {
        int n;
        int i[RG_SETS], sq[RG_SETS], ab[RG_SETS];
    };
    struct Idx {
        int n;
        int i[RG_SETS];
    };
    auto idx_load = [&](int D) {
        Idx X;
        X.n = 0;
#pragma unroll
        for (int k = 0; k < RG_SETS; k++) X.i[k] = 1;
        if (D < 6 || D > N - 1) return X;
        const int od = off(D, N);
        X.n = uni(L.cn[D]);
        const int i0 = L.cl[od];
#pragma unroll
        for (int k = 0; k < RG_SETS; k++) {
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
        for (int k = 0; k < RG_SETS; k++) {
            Q.i[k] = X.i[k];
            Q.sq[k] = 0;
            Q.ab[k] = 0;
            if (k * WAVE >= Q.n) continue;
            const int i = X.i[k], j = i + D;
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
        for (int k = 0; k < RG_SETS; k++) {
            P.w1[k] = 0;
            P.mmo[k] = P.mo[k] = P.m23[k] = P.t11[k] = P.t12[k] = P.t21[k] = P.t22[k] = 0.f;
            if (k * WAVE >= Q.n) continue;
            const bool v = k * WAVE + lane < Q.n;
            const int i = Q.i[k], sqk = Q.sq[k];
            const int ty = sqk & 15, si1 = (sqk >> 4) & 15, sj1 = (sqk >> 8) & 15, si2 = (sqk >> 12) & 15,
                      sj2 = (sqk >> 16) & 15;
            const int oc = ty * 25 + si1 * 5 + sj1;
            const int A = Q.ab[k] & 255, Bq = Q.ab[k] >> 8;
            // the 1x1..2x2 inner codes: diagonals D-4 .. D-6 are in the ring
            auto t2of = [&](int n1, int n2) { return (L.cc[rgo(D - 2 - n1 - n2, RS) + i + n1] * 41) >> 10; };
            if (umax >= 2) P.t11[k] = T.int11[ty][t2of(1, 1)][si1][sj1];
            if (umax >= 3) {
                P.t12[k] = T.int21[ty][t2of(1, 2)][si1][sj2][sj1];
                P.t21[k] = T.int21[t2of(2, 1)][ty][sj1][si1][si2];
            }
            if (umax >= 4) P.t22[k] = T.int22[ty][t2of(2, 2)][si1][si2][sj2][sj1];
            const bool mkc = A < umax || Bq < umax;
            P.w1[k] = i | (ty << 8) | (A << 11) | (Bq << 19) | (mkc ? (1 << 27) : 0) | (v ? (1 << 28) : 0);
            P.mmo[k] = L.dt[DT_MMI + oc];
            P.mo[k] = ct[CT_ONEN + oc] * P.mmo[k];
            P.m23[k] = ct[CT_M23O + oc];
        }
        return P;
    };
    auto rec_store = [&](int D, const Pend &P) {
#pragma unroll
        for (int k = 0; k < RG_SETS; k++) {
            if (k * WAVE >= P.n) break;
            float *r = L.rec + (((D & 1) * RG_SETS + k) * RG_RF) * WAVE + lane;
            r[0] = __int_as_float(P.w1[k]);
            r[WAVE] = P.mmo[k];
            r[2 * WAVE] = P.mo[k];
            r[3 * WAVE] = P.m23[k];
            r[4 * WAVE] = P.t11[k];
            r[5 * WAVE] = P.t12[k];
            r[6 * WAVE] = P.t21[k];
            r[7 * WAVE] = P.t22[k];
        }
        if (lane == 0) L.rcnt[D & 1] = P.n;
    };
    Pend pend;
    Seq seqp;
    Idx idxp;
    if (wid == RG_WR) {
        rec_store(4, rec_load(4, seq_load(4, idx_load(4))));
        pend = rec_load(5, seq_load(5, idx_load(5)));
        seqp = seq_load(6, idx_load(6));
        idxp = idx_load(7);
    }
    if (ph >= 0) {   // diagonal 4 before the sweep, diagonal 5's restored values in flight
        rload(4, ph);
        prep(4, ph);
        vm_drain();
        rload(5, ph);
    }
    __syncthreads();

    // Q: exterior-stem factors of column j (cells (k, j), k <= j - 4, three
    // lane-sets): INVMM(code) * ext(type, S[k-1], S[j+1]), gathered a step ahead
    float qf[RG_SETS] = {0.f, 0.f, 0.f}, qv[RG_SETS] = {0.f, 0.f, 0.f};
    int qcol = -1;   // the column qf / qv hold
    auto qload = [&](int j) {   // column j of qb from the slot / scratch, and its factors
        qcol = -1;
        if (j < 5 || j > N || (incr && j < m_lo - 1)) return;
        qcol = j;
        const int sjp = (j < N) ? S[j + 1] : 5;
        const int sj = S[j];
#pragma unroll
        for (int h = 0; h < RG_SETS; h++) {
            const int kk = 1 + h * WAVE + lane;
            const bool ok = kk <= j - 4;
            const int k = ok ? kk : 1;
            const int ty = ptype(S[k], sj);
            const int code = rtype(ty) * 25 + S[j + 1] * 5 + S[k - 1];   // the cell's inner code (S wraps)
            const float e = L.dt[DT_EXT + ty * 36 + ((k > 1) ? S[k - 1] : 5) * 6 + sjp];
            qf[h] = ok ? ct[CT_INVMM + code] * e : 0.f;
            qv[h] = ok && h * WAVE < j - 4 ? qbg[off(j - k, N) + k - 1] : 0.f;
        }
    };
    const int s_end = N + 3;   // Q finishes q5[N] three steps after column N is final
    RSTAMP(0);   // setup
    if (wid < RG_NB) {
        switch (wid) {
            // (A/B knob RG_PART: sizes moved off block 4, the busiest in the stamps,
            // profiles/r06u_pf_ring_stamps.txt)
#if RG_PART == 1   // 13 -> block 0, 0 -> block 1
            case 0: rb_sweep<5, 22, 12, 11, 13>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 1: rb_sweep<4, 21, 19, 10, 0>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 4: rb_sweep<29, 27, 16, -1, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            default: rb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
#elif RG_PART == 2   // 16 -> block 0
            case 0: rb_sweep<5, 22, 12, 11, 16>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 1: rb_sweep<4, 21, 19, 10, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 4: rb_sweep<29, 27, 13, 0, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            default: rb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
#elif RG_PART == 3   // 13 -> block 6, 0 -> block 1
            case 0: rb_sweep<5, 22, 12, 11, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 1: rb_sweep<4, 21, 19, 10, 0>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 4: rb_sweep<29, 27, 16, -1, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            default: rb_sweep<24, 25, 23, 15, 13>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
#else
            case 0: rb_sweep<5, 22, 12, 11, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 1: rb_sweep<4, 21, 19, 10, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 4: rb_sweep<29, 27, 16, 13, 0>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            default: rb_sweep<24, 25, 23, 15, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
#endif
            case 2: rb_sweep<3, 20, 18, 8, 6>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 3: rb_sweep<28, 26, 1, 9, 7>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
            case 5: rb_sweep<30, 2, 17, 14, -1>(L, XS, N, lane, wid, constrained, s_end RG_STP_ARGS); break;
        }
    } else {
        __builtin_amdgcn_s_setprio(2);
        // one sweep instance per role (round 6, as pf_cells.hip): the shared loop
        // kept every role's values live (65 SGPR spill reads / writes per step)
        auto sweep = [&](auto role_c) __attribute__((always_inline)) {
        constexpr int ROLE = decltype(role_c)::value;   // 0 M, 1 F, 2 Q, 3 R
        for (int s = 4; s <= s_end; s++) {
            if constexpr (ROLE == 0) {
                // ---------------- M: qm items of span sq = s - 2 (pf_cells.hip)
                const int sq = s - 2;
                if (sq >= 4 && sq <= N - 3) {
                    const int lo = qlo(sq), n = qhi(sq) - lo + 1;
                    int K = 16;
                    while (K > 1 && (N - sq) * K > RG_NMW * WAVE) K >>= 1;
                    const int mw = rg_mw(wid);
                    const int k = lane & (K - 1);
                    // K and the split ranges follow the full fold's item count, so a
                    // refold sums every item as a fold from scratch does (n <= N - sq
                    // <= RG_NMW * WAVE / K: one round)
                    const int ipw = WAVE / K;
                    if (mw * ipw < n) {
                        const int item = mw * ipw + lane / K;
                        const bool valid = item < n;
                        const int i = lo + (valid ? item : n - 1);
                        const int jb = i + sq, T = sq - 4;
                        // split points t = 5..T; the unpaired part is the column recursion
                        // U(i, jb) = qm1(i, jb) + [up_i >= 1] (expMLbase sigma) U(i+1, jb),
                        // U of span sq - 1 kept by the Q wave (pf_cells.hip)
                        const int nb = T - 4;
                        const int tch = nb > 0 ? (nb + K - 1) / K : 0;
                        const int t0 = 5 + k * tch, t1 = min(T, t0 + tch - 1);
                        const float *pq = L.q1 + colb(jb) + i - 1;
                        const float *pr = L.qm + rowb(i, N) - 5;
                        const bool up1 = sq >= 5 && (!constrained || L.up[i] >= 1);
                        const float u1 = up1 ? L.uc[((sq - 1) & 1) * NP + jb] : 0.f;
                        const float q0 = pq[0];
                        float A = 0.f, A1 = 0.f;
                        for (int t = t0; t <= t1; t += 2) {   // pairs: even offsets in A, odd in A1
                            const float qa = pq[t], qn = pq[t + 1], ra = pr[t], rn = pr[t + 1];
                            A = fmaf(ra, qa, A);
                            A1 = fmaf(rn, t + 1 <= t1 ? qn : 0.f, A1);
                        }
                        A += A1;
                        if (K >= 2) A = dpp_add<0xb1>(A);
                        if (K >= 4) A = dpp_add<0x4e>(A);
                        if (K >= 8) A = dpp_add<0x114>(A);
                        if (K >= 16) A = dpp_add<0x118>(A);
                        if (valid && k == (K >= 8 ? K - 1 : 0)) {
                            L.qm[rowb(i, N) + sq - 4] = A + fmaf(mlbase_sig, u1, q0);
                            L.mla[(sq & 1) * NP + i] = A;
                        }
                    }
                }
                if (ph >= 0) {
                    // the prep of lane-set ph of diagonal s + 1 (its restored values were
                    // loaded last step); the drain first completes last step's prep
                    // stores (read by Q two steps on) and loads, a step old by now
                    RSTAMP(5);
                    vm_drain();
                    prep(s + 1, ph);
                    RSTAMP(6);
                    rload(s + 2, ph);   // in flight across the barrier
                }
            } else if constexpr (ROLE == 1) {
                vm_drain();        // last step's finalised cells (Q loads them this step)
                // ---------------- F: the changed cells of diagonal e = s - 1
                const int e = s - 1;
                if (e >= 4 && e <= N - 1) {
                    const int lo = clo(e), hi = chi(e);
                    const int ro = rgo(e, RS), od = off(e, N);
                    for (int i0 = lo; i0 <= hi; i0 += WAVE) {
                        const int i = i0 + lane;
                        if (i > hi) break;
                        const int j = i + e;
                        const int ce = ro + i - 1, c1 = colb(j) + i - 1;
                        const float init = L.qb[ce];
                        const float stem = L.q1[c1];
                        const bool upj = e >= 5 && L.up[j] >= 1;
                        const float prev = upj ? L.q1[colb(j - 1) + i - 1] : 0.f;
                        if (__float_as_uint(init) != 0x80000000u) {
                            const int ty = ptype(S[i], S[j]);
                            const float mlcl = mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
                            float a_int = 0.f;
                            if (e >= 6) {
                                const float *pp = L.part + ((e & 1) * RG_SETS + ((i - 1) >> 6)) * RG_NB * WAVE +
                                                  ((i - 1) & (WAVE - 1));
#pragma unroll
                                for (int b = 0; b < RG_NB; b++) a_int += pp[b * WAVE];
                            }
                            const float ml = e - 2 >= 4 ? L.mla[((e - 2) & 1) * NP + i + 1] : 0.f;
                            const float qb = a_int + init + ml * mlcl;
                            const float mmc = L.dt[DT_MMI + L.cc[ce]];
                            const float fin = qb * mmc + 0.f;   // never the mark (-0)
                            L.qb[ce] = fin;
                            qbg[od + i - 1] = fin;
                            L.q1[c1] = fmaf(qb, stem, prev * mlbase_sig);
                        } else {
                            L.q1[c1] = prev * mlbase_sig;
                        }
                    }
                }
            } else if constexpr (ROLE == 2) {
                // ---------------- Q: q5[j], j = s - 3, from column j loaded last step
                const int j = s - 3;
                if (j >= 4 && j <= N && (!incr || j >= m_lo - 1)) {
                    float acc = 0.f;
                    if (qcol == j) {
#pragma unroll
                        for (int h = 0; h < RG_SETS; h++) {
                            if (h * WAVE >= j - 4) break;
                            const int kk = 1 + h * WAVE + lane;
                            const int k = kk <= j - 4 ? kk : 1;
                            acc = fmaf(L.q5[k - 1] * qv[h], qf[h], acc);
                        }
                    }
                    acc = wave_sum_dpp(acc);
                    if (lane == 0) L.q5[j] = (L.up[j] >= 1 ? L.q5[j - 1] * sig1 : 0.f) + acc;
                }
                RSTAMP(5);         // q5
                {   // U(i, jb) of span sq = s - 2 for every cell (M reads it next step)
                    const int sq = s - 2;
                    if (sq >= 4 && sq <= N - 4) {
                        for (int i = 1 + lane; i <= N - sq; i += WAVE) {
                            const int jb = i + sq;
                            const bool up1 = sq >= 5 && (!constrained || L.up[i] >= 1);
                            const float u1 = up1 ? L.uc[((sq - 1) & 1) * NP + jb] : 0.f;
                            L.uc[(sq & 1) * NP + jb] = fmaf(mlbase_sig, u1, L.q1[colb(jb) + i - 1]);
                        }
                    }
                }
                // column s - 2 is final: its last cell, (1, s-2), was finalised two steps
                // ago and its store drained by F at the start of the last step
                qload(s - 2);
            } else {
                vm_drain();        // last step's prep stores and loads (the record loads are a step old)
                prep(s + 1, 2);
                rload(s + 2, 2);
                rec_store(s + 1, pend);
                pend = rec_load(s + 2, seqp);
                seqp = seq_load(s + 3, idxp);
                idxp = idx_load(s + 4);
            }
            RSTAMP(3);   // the role's step work
            lds_barrier();
            RSTAMP(7);   // barrier
        }
        };
        if (rg_mw(wid) >= 0) sweep(std::integral_constant<int, 0>{});
        else if (wid == RG_WF) sweep(std::integral_constant<int, 1>{});
        else if (wid == RG_WQ) sweep(std::integral_constant<int, 2>{});
        else sweep(std::integral_constant<int, 3>{});   // RG_WR
    }
    __syncthreads();
    RSTAMP(4);
#ifdef ADX_STAMP
    if (lane == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_stamps_r[wid][k], st_acc[k]);
#endif
    // ---- the proposal's qm / qm1 to the slot, diagonal-major (qb is there already)
    if (dst) {
        for (int D = 4 + wid; D <= N - 1; D += RG_NW) {
            const int od = off(D, N);
            for (int i = 1 + lane; i <= N - D; i += WAVE) {
                dst[Cs + od + i - 1] = L.qm[rowb(i, N) + D - 4];
                dst[2 * Cs + od + i - 1] = L.q1[colb(i + D) + i - 1];
            }
        }
        for (int k = tid; k <= N; k += RG_NT) dst[3 * Cs + k] = L.q5[k];
    }
    if (tid == 0) {   // ensemble energy -kT (ln Z_scaled - N ln sigma), as vrna_pf (float)
        const float z = L.q5[N];
        const float g = float(-XS->kT * (log(double(z)) - N * XS->log_sigma));
        gout[size_t(w) * ka.n_variants + vh] = g;
    }
}

}  // namespace

// LDS bytes of the ring PF kernel for this workload (0: not covered)
size_t pf_ring_lds(const KArgs &ka) {
    if (ka.mode != 0 || ka.Nmax < RG_NMIN || ka.Nmax > RG_NMAX) return 0;
    const size_t b = RgLay(ka.Nmax).BYTES;
    return b + 256 <= 160 * 1024 ? b : 0;
}
// floats of per-workgroup qb scratch a stateless launch needs
size_t pf_ring_scratch_floats(const KArgs &ka, int W) {
    return size_t(W) * 2 * ka.n_groups2 * size_t(ka.cells);
}

hipError_t launch_pf_ring(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, float *gout,
                          float *qscr, hipStream_t stream) {
    const size_t lds = pf_ring_lds(ka);
    if (lds == 0 || (!ka.tab && !qscr)) return hipErrorInvalidValue;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(pf_ring_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(pf_ring_kernel, dim3(W * 2 * ka.n_groups2), dim3(RG_NT), lds, stream, ka, ka.X, seqs, W, mask,
                       gout, qscr);
    return hipGetLastError();
}

}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_ring(unsigned long long *out, int reset) {  // [16][8]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_r), sizeof(adx::g_stamps_r)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_r), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
