// gfx950 outside pass (base-pair probabilities, SURVEY.md A16 / BASELINE
// configs 3-4) with lanes = cells: the adjoint of the inside recursions of
// kernels.hip pf_group, in gather form and descending span order -- the same
// equations as kernels.hip outside() (oracle/fold.c orc_bppm is the scatter
// form of the sweep), mapped the way mfe_cells.hip maps the MFE:
//
//   * one workgroup (16 waves) per (walker, unconstrained fold with pair
//     terms); the fold's inside tables are NOT recomputed: score_kernel has
//     just written them to the walker's next incremental slot (KArgs::tab), and
//     they are loaded from there into LDS, all diagonal-major;
//   * one anti-diagonal per step, ONE barrier per step; a lane holds one cell
//     (i, i+d), so every interior-loop shape (n1, n2) is one LDS read per lane of
//     the outer cell (i-1-n1, j+1+n2) at a per-lane base plus an immediate
//     offset, no cross-lane reduction.  The 496 shapes are split by loop size
//     over 12 waves (B); waves 12-15 sum the multiloop adjoints (M); the next
//     step finalizes the cell (F).
//
//   q5b[m]    = sigma q5b[m+1] + sum_j q5b[j] qb(m+1,j) ext(m+1,j)   (before the sweep)
//   qmb(i,j)  = sum_{l >= j+5} Y(i,l) qm1(j+1,l)                      (M)
//   r2(i,j)   = sum_{ip <= i-5} Y(ip,j) qm(ip,i-1)                     (M)
//   R(i,j)    = pw1 (qmb(i-1,j) + R(i-1,j))     [= sum_ip qmb(ip,j) pw(i-ip); pw geometric]
//   qm1b(i,j) = qmb + R + r2 + expMLbase sigma qm1b(i,j+1)
//   qbb(i,j)  = sum_{outer (a,b), loop <= 30} qbb(a,b) F_int + q5b[j] q5[i-1] ext + qm1b stemM   (B, F)
//   Y(i,j)    = qmb(i,j) + X(i,j),  X(i+1,j-1) = qbb(i,j) MLclosing stemM(rev)
//   P(i,j)    = qb(i,j) qbb(i,j) / Z
//
// Covered: unconstrained folds (the pair terms' folds are the conditions'
// unconstrained folds, adx_api.cpp), N <= 128 (LDS); everything else takes
// kernels.hip bppm_kernel.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {
namespace {

constexpr int OX_NW = 16;             // waves per workgroup
constexpr int OX_NT = OX_NW * WAVE;
constexpr int OX_NB = 12;             // interior-loop blocks (waves 0..11)
constexpr int OX_WIN = 32;            // qbb window: spans d+2 .. d+32 are read at step d
constexpr int OX_PAD = 32;            // zero cells in front of each window row (outer a >= i-31)
constexpr int OX_MAXP = 64;           // requested pairs of one fold kept in LDS
constexpr int OX_NMAX = 128;

// LDS carve for folded length N (runtime; the host sizes the launch with it)
struct OxLay {
    int C, NP, RL;
    size_t Y, QM, QM1, QW, OW, PART, MLP, RQ, RR, R1, Q5, Q5B, PM, CT, DT, PD, S, MT, BYTES;
    __host__ __device__ static size_t a16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ explicit OxLay(int N) {
        C = ((N - 4) * (N - 3)) / 2;
        NP = N + 2;
        RL = N + 2 * OX_PAD;
        size_t o = 0;
        Y = o;    o += a16(size_t(C) * 4);                       // Y (qbm_in before the sweep)
        QM = o;   o += a16(size_t(C) * 4);                       // inside qm, diagonal-major
        QM1 = o;  o += a16(size_t(C) * 4);                       // inside qm1, diagonal-major
        QW = o;   o += a16(size_t(OX_WIN) * RL * 4);             // qbb * mismatchI(outer) window
        OW = o;   o += a16(size_t(OX_WIN) * RL);                 // outer codes window
        PART = o; o += a16(size_t(2) * 2 * OX_NB * WAVE * 4);   // [parity][lane-set][block][lane]
        MLP = o;  o += a16(size_t(2) * 4 * WAVE * 4);           // [parity][M wave][lane]
        RQ = o;   o += a16(size_t(2) * NP * 4);                  // qmb ring [parity][i]
        RR = o;   o += a16(size_t(2) * NP * 4);                  // R ring
        R1 = o;   o += a16(size_t(2) * NP * 4);                  // qm1b ring
        Q5 = o;   o += a16(size_t(NP) * 4);
        Q5B = o;  o += a16(size_t(NP) * 4);
        PM = o;   o += a16(size_t(NP) * 4);                      // motif site weights
        CT = o;   o += a16(size_t(CT_SIZE) * 4);
        DT = o;   o += a16(size_t(DT_EXT + 288) * 4);            // MMI, MLS, EXT
        PD = o;   o += a16(size_t(OX_MAXP) * 8);                 // requested pairs: qb qbb / Z
        S = o;    o += a16(size_t(NP) + 8);
        MT = o;   o += a16(size_t(NP));                          // motif site flags
        BYTES = o;
    }
};

struct OxL {
    float *Y, *qm, *qm1, *qw, *part, *mlp, *rq, *rr, *r1, *q5, *q5b, *pm, *ct, *dt;
    uint8_t *ow, *S, *mat;
    double *pd;
    int RL, NP;
};

__device__ __forceinline__ int wslot(int D) { return D & (OX_WIN - 1); }

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

// Shapes of loop size U for the lane's cell; qw / ow: this lane's window row of
// the outer span d + 2 + U at outer a = i - 1 - U (n1 = U), so shape n1 reads
// offset U - n1.
template <int U>
__device__ __forceinline__ void oshape(const OxL &L, const DevScaled *__restrict__ XS, const OxCell &c,
                                       const float *qw, const uint8_t *ow, int ty2, float &g, float &sp) {
    const float *ct = L.ct;
#pragma unroll
    for (int n1 = 0; n1 <= U; n1++) {
        const int n2 = U - n1;
        const float v = qw[U - n1];
        const int k = okind(n1, n2);
        if (k < 0) {
            g = fmaf(v, XS->fgen[(U - 6) * FG_ROW + n1 - 2], g);
        } else {
            const int oc = ow[U - n1];
            float f;
            if (k == TK_STK || k == TK_B1) {
                f = ct[CT_INVMM + oc] * ct[CT_STK + ((oc * 41) >> 10) * 8 + ty2] * XS->ctab[CT_FSM + (k == TK_B1 ? 1 : 0)];
            } else if (k == TK_BUL) {
                f = ct[CT_BUL + oc] * (c.tau_in * XS->ctab[CT_FB + U]);
            } else if (k == TK_1N) {
                f = ct[CT_ONEN + oc] * (c.mo_in * XS->ctab[CT_F1N + U - 1]);
            } else if (k == TK_M23) {
                f = ct[CT_INVMM + oc] * ct[CT_M23O + oc] * (c.m23_in * XS->ctab[CT_FSM + 5]);
            } else {
                const float tv = k == TK_I11 ? c.t11 : k == TK_I12 ? c.t12 : k == TK_I21 ? c.t21 : c.t22;
                const int fs = k == TK_I11 ? 2 : k == TK_I22 ? 4 : 3;
                f = ct[CT_INVMM + oc] * (tv * XS->ctab[CT_FSM + fs]);
            }
            sp = fmaf(v, f, sp);
        }
    }
}

// one loop size of a block: skipped past the step's umax (uniform)
#define OX_U(U)                                                                                   \
    if ((U) <= umax) {                                                                            \
        const int o = wslot(d + 2 + (U)) * L.RL + OX_PAD + c.i - 2 - (U);                         \
        oshape<(U)>(L, XS, c, L.qw + o, L.ow + o, ty2, g, sp);                                    \
    }

// blocks of loop sizes of about equal cost (generic shape ~2 instructions, a
// special ~9); the 1x1..2x2 table shapes (u = 2, 3, 4) share blocks with large
// loops so the table loads issued at the block start land meanwhile
__device__ __forceinline__ void oblock(int b, const OxL &L, const DevScaled *__restrict__ XS, const OxCell &c,
                                       int d, int umax, int ty2, float &g, float &sp) {
    switch (b) {
        case 0: OX_U(8) OX_U(30) break;
        case 1: OX_U(9) OX_U(29) break;
        case 2: OX_U(10) OX_U(28) break;
        case 3: OX_U(11) OX_U(27) break;
        case 4: OX_U(12) OX_U(26) break;
        case 5: OX_U(25) OX_U(5) OX_U(4) break;
        case 6: OX_U(7) OX_U(13) OX_U(24) break;
        case 7: OX_U(6) OX_U(14) OX_U(23) break;
        case 8: OX_U(22) OX_U(15) OX_U(3) break;
        case 9: OX_U(21) OX_U(16) OX_U(2) break;
        case 10: OX_U(1) OX_U(17) OX_U(20) break;
        default: OX_U(0) OX_U(18) OX_U(19) break;
    }
}
constexpr unsigned OX_TABLE_BLOCKS = (1u << 5) | (1u << 8) | (1u << 9);   // blocks with u = 4 / 3 / 2

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

// One workgroup per (walker, outside variant).  pair_p: [W][n_pairs].
__global__ void __launch_bounds__(OX_NT, 1)
outside_cells_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, const int *mask,
                     double *pair_p, int sp_score) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int w = blockIdx.x / ka.n_bvars, bv = blockIdx.x % ka.n_bvars;
    if (w >= W) return;
    if (mask && mask[w] != 1) return;
    const int v = ka.bvars[bv];
    const DevVariant V = ka.variants[v];
    const int N = uni(V.N);
    const OxLay Y(N);
    OxL L;
    L.Y = reinterpret_cast<float *>(smem + Y.Y);
    L.qm = reinterpret_cast<float *>(smem + Y.QM);
    L.qm1 = reinterpret_cast<float *>(smem + Y.QM1);
    L.qw = reinterpret_cast<float *>(smem + Y.QW);
    L.ow = reinterpret_cast<uint8_t *>(smem + Y.OW);
    L.part = reinterpret_cast<float *>(smem + Y.PART);
    L.mlp = reinterpret_cast<float *>(smem + Y.MLP);
    L.rq = reinterpret_cast<float *>(smem + Y.RQ);
    L.rr = reinterpret_cast<float *>(smem + Y.RR);
    L.r1 = reinterpret_cast<float *>(smem + Y.R1);
    L.q5 = reinterpret_cast<float *>(smem + Y.Q5);
    L.q5b = reinterpret_cast<float *>(smem + Y.Q5B);
    L.pm = reinterpret_cast<float *>(smem + Y.PM);
    L.ct = reinterpret_cast<float *>(smem + Y.CT);
    L.dt = reinterpret_cast<float *>(smem + Y.DT);
    L.pd = reinterpret_cast<double *>(smem + Y.PD);
    L.S = reinterpret_cast<uint8_t *>(smem + Y.S);
    L.mat = reinterpret_cast<uint8_t *>(smem + Y.MT);
    L.RL = Y.RL;
    L.NP = Y.NP;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
    const int C = Y.C, NP = Y.NP;
    const DevTables &T = *ka.T;

    // ---- the proposal's inside tables (score_kernel's P = sp_score layout, kernels.hip Inc)
    const size_t B = 3 * size_t(ka.cells) + size_t(ka.Nmax) + 2;
    size_t go = size_t(v) * B;
    if (sp_score == 2) {
        for (int g = 0; g < ka.n_groups2; g++) {
            if (ka.groups2[2 * g] == v) { go = size_t(g) * 2 * B; break; }
            if (ka.groups2[2 * g + 1] == v) { go = size_t(g) * 2 * B + B; break; }
        }
    }
    const int cur = ka.cur_slot[w];
    const float *src = ka.tab + size_t(w) * 2 * ka.tab_slot + size_t(1 - cur) * ka.tab_slot + go;
    const size_t Cs = size_t(ka.cells);   // the slot's table stride (Nmax cells)

    // sequence (kernels.hip pf_group: contexts, ViennaRNA S1 wrap)
    {
        const uint8_t *bef = nullptr, *aft = nullptr;
        int blen = 0;
        if (V.ctx >= 0) {
            bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
            blen = ka.ctx_off[4 * V.ctx + 1];
            aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
        }
        const uint8_t *raw = seqs + size_t(w) * ka.Nraw;
        for (int k = tid; k < NP; k += OX_NT) {
            uint8_t s = 0;
            if (k >= 1 && k <= N) {
                const int pp = k - 1;
                if (pp < blen) s = bef[pp];
                else if (pp < blen + ka.Nraw) s = raw[pp - blen];
                else s = aft[pp - blen - ka.Nraw];
            }
            L.S[k] = s;
        }
    }
    for (int k = tid; k < CT_SIZE; k += OX_NT) L.ct[k] = XS->ctab[k];
    for (int k = tid; k < 200; k += OX_NT) {
        L.dt[DT_MMI + k] = (&T.mmI[0][0][0])[k];
        L.dt[DT_MLS + k] = (&T.mlstem[0][0][0])[k];
    }
    for (int k = tid; k < 288; k += OX_NT) L.dt[DT_EXT + k] = (&T.ext[0][0][0])[k];
    // inside tables: qbm (diagonal-major, as stored) into the Y region for the
    // exterior adjoint, qm (row-major) and qm1 (column-major) transposed
    for (int D = 4; D <= N - 1; D++) {
        const int od = off(D, N);
        for (int r = tid; r < N - D; r += OX_NT) {
            const int i = r + 1, j = i + D;
            L.Y[od + r] = src[od + r];
            L.qm[od + r] = src[Cs + rowb(i, N) + D - 4];
            L.qm1[od + r] = src[2 * Cs + colb(j) + i - 1];
        }
    }
    for (int k = tid; k <= N; k += OX_NT) L.q5[k] = src[3 * Cs + k];
    for (int k = tid; k < OX_WIN * L.RL; k += OX_NT) {
        L.qw[k] = 0.f;
        L.ow[k] = 0;
    }
    for (int k = tid; k < 2 * NP; k += OX_NT) L.rq[k] = L.rr[k] = L.r1[k] = 0.f;
    for (int k = tid; k < NP; k += OX_NT) { L.q5b[k] = 0.f; L.pm[k] = 0.f; L.mat[k] = 0; }
    for (int k = tid; k < OX_MAXP; k += OX_NT) L.pd[k] = 0.0;
    __syncthreads();
    if (tid == 0) {
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
    }
    __syncthreads();
    const uint8_t *S = L.S;
    const float *ct = L.ct;
    const float Z = L.q5[N];
    const bool motif = V.motif != 0 && XS->motif_len > 0;
    const int mL = XS->motif_len;

    // ---- exterior adjoint q5b (one wave, sequential in m; kernels.hip outside())
    if (wid == 0) {
        const float sig1 = XS->sig[1];
        if (lane == 0) L.q5b[N] = 1.f;
        float nxt = 1.f;
        for (int m = N - 1; m >= 0; m--) {
            const int k = m + 1;
            float acc = 0.f;
            for (int j = k + 4 + lane; j <= N; j += WAVE) {
                const int ty = ptype(S[k], S[j]);
                const int cc = rtype(ty) * 25 + S[j + 1] * 5 + S[k - 1];
                const float e = L.dt[DT_EXT + ty * 36 + ((k > 1) ? S[k - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
                acc = fmaf(L.q5b[j] * L.Y[off(j - k, N) + k - 1], ct[CT_INVMM + cc] * e, acc);
            }
            const float val = nxt * sig1 + wave_sum_f(acc);
            if (lane == 0) L.q5b[m] = val;
            nxt = val;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    // motif sites (unconstrained: the sequence alone decides)
    if (motif && wid == 1) {
        for (int o = lane + 1; o + mL - 1 <= N; o += WAVE) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) ok = S[o + k] == XS->motif_code[k];
            L.mat[o] = ok ? 1 : 0;
        }
    }
    __syncthreads();
    for (int k = tid; k < C; k += OX_NT) L.Y[k] = 0.f;
    __syncthreads();

    const float mlbase_sig = XS->mlbase_sig, mlclosing = XS->mlclosing, pw1 = XS->pwml[1];
    const float eTAU = XS->ctab[CT_FSM + 6];

    // ---- the sweep: step d runs B and M of diagonal d and F of diagonal d + 1
    for (int d = N - 1; d >= 3; d--) {
        const int nls = d >= 4 ? (N - d + WAVE - 1) / WAVE : 0;   // lane-sets of diagonal d
        const int par = d & 1;
        if (wid < OX_NB) {
            // ---------------- B: interior-loop gather of diagonal d (outer spans d+2 .. d+2+umax)
            const int umax = min(30, N - 3 - d);
            for (int ls = 0; ls < nls; ls++) {
                int i = 1 + ls * WAVE + lane;
                const bool valid = i <= N - d;
                if (!valid) i = N - d;
                const int j = i + d;
                const int ty = ptype(S[i], S[j]);
                const bool pr = valid && ty != 0;
                float *pout = L.part + ((par * 2 + ls) * OX_NB + wid) * WAVE + lane;
                if (umax < 0 || __ballot(pr) == 0) {   // no outer loop fits (or nothing pairs)
                    *pout = 0.f;
                    continue;
                }
                OxCell c;
                c.i = i;
                const int ty2 = rtype(ty);
                const int cc = ty2 * 25 + S[j + 1] * 5 + S[i - 1];
                c.mmin = L.dt[DT_MMI + cc];
                c.tau_in = ty2 > 2 ? eTAU : 1.f;
                c.mo_in = ct[CT_ONEN + cc] * c.mmin;
                c.m23_in = ct[CT_M23O + cc];
                c.t11 = c.t12 = c.t21 = c.t22 = 0.f;
                if ((OX_TABLE_BLOCKS >> wid) & 1) {
                    auto Sc = [&](int x) { return int(S[x < 0 ? 0 : (x > N + 1 ? N + 1 : x)]); };
                    if (umax >= 2) {
                        const int t1 = ptype(Sc(i - 2), Sc(j + 2));
                        c.t11 = T.int11[t1][ty2][Sc(i - 1)][Sc(j + 1)];
                    }
                    if (umax >= 3) {
                        const int ta = ptype(Sc(i - 2), Sc(j + 3)), tb = ptype(Sc(i - 3), Sc(j + 2));
                        c.t12 = T.int21[ta][ty2][Sc(i - 1)][Sc(j + 1)][Sc(j + 2)];
                        c.t21 = T.int21[ty2][tb][Sc(j + 1)][Sc(i - 2)][Sc(i - 1)];
                    }
                    if (umax >= 4) {
                        const int t1 = ptype(Sc(i - 3), Sc(j + 3));
                        c.t22 = T.int22[t1][ty2][Sc(i - 2)][Sc(i - 1)][Sc(j + 1)][Sc(j + 2)];
                    }
                }
                float g = 0.f, sp = 0.f;
                oblock(wid, L, XS, c, d, umax, ty2, g, sp);
                *pout = fmaf(g, c.mmin, sp);
            }
        } else {
            // ---------------- M: multiloop adjoint sums of diagonal d
            const int mw = wid - OX_NB;                 // 0, 1: qmb; 2, 3: r2
            const bool two = nls == 2;
            const int ls = two ? (mw & 1) : 0;
            if (d >= 4 && ls < nls) {
                int i = 1 + ls * WAVE + lane;
                const bool valid = i <= N - d;
                if (!valid) i = N - d;
                const int j = i + d;
                float acc = 0.f;
                if (mw < 2) {
                    // qmb: t = 0 .. N-j-5, Y(i, j+5+t) = diag d+5+t, qm1(j+1, j+5+t) = diag 4+t
                    const int lim = N - j - 5;
                    const int tmax = N - (1 + ls * WAVE + d) - 5;           // lane-set's first cell
                    const int h = two ? tmax + 1 : (tmax + 2) / 2;
                    const int t0 = (two || mw == 0) ? 0 : h, t1 = two ? tmax + 1 : (mw == 0 ? h : tmax + 1);
                    int ay = off(d + 5 + t0, N) + i - 1, aq = off(4 + t0, N) + j;
                    for (int t = t0; t < t1; t++) {
                        if (t <= lim) acc = fmaf(L.Y[ay], L.qm1[aq], acc);
                        ay += N - (d + 5 + t);
                        aq += N - (4 + t);
                    }
                } else {
                    // r2: t = 5 .. i-1, Y(i-t, j) = diag d+t, qm(i-t, i-1) = diag t-1
                    const int imax = min(N - d, (ls + 1) * WAVE);
                    const int tmax = imax - 1;
                    const int h = two ? tmax + 1 : (5 + tmax + 2) / 2;
                    const int t0 = (two || mw == 2) ? 5 : h, t1 = two ? tmax + 1 : (mw == 2 ? h : tmax + 1);
                    if (t0 < t1) {
                        int ay = off(d + t0, N) + i - t0 - 1, aq = off(t0 - 1, N) + i - t0 - 1;
                        for (int t = t0; t < t1; t++) {
                            if (t <= i - 1) acc = fmaf(L.Y[ay], L.qm[aq], acc);
                            ay += N - (d + t) - 1;
                            aq += N - (t - 1) - 1;
                        }
                    }
                }
                L.mlp[(par * 4 + mw) * WAVE + lane] = acc;
            }
            // ---------------- F: finalize diagonal e = d + 1 (lane-set mw on wave 12 + mw)
            const int e = d + 1;
            const int nle = (N - e + WAVE - 1) / WAVE;
            if (e <= N - 1 && mw < 2 && mw < nle) {
                const int fl = mw;
                const int pe = e & 1, pn = (e + 1) & 1;
                const int i = 1 + fl * WAVE + lane;
                if (i <= N - e) {
                    const int j = i + e;
                    const bool te = nle == 2;
                    const float *mp = L.mlp + pe * 4 * WAVE;
                    const float qmbv = te ? mp[fl * WAVE + lane] : mp[lane] + mp[WAVE + lane];
                    const float r2 = te ? mp[(2 + fl) * WAVE + lane] : mp[2 * WAVE + lane] + mp[3 * WAVE + lane];
                    const float R = i >= 2 ? pw1 * (L.rq[pn * NP + i - 1] + L.rr[pn * NP + i - 1]) : 0.f;
                    const float chain = j < N ? mlbase_sig * L.r1[pn * NP + i] : 0.f;
                    const float qm1b = qmbv + R + r2 + chain;
                    L.rq[pe * NP + i] = qmbv;
                    L.rr[pe * NP + i] = R;
                    L.r1[pe * NP + i] = qm1b;
                    const int ce = off(e, N) + i - 1;
                    L.Y[ce] += qmbv;   // X(i, j) was stored two diagonals ago
                    const int ty = ptype(S[i], S[j]);
                    const int oc = ty * 25 + S[i + 1] * 5 + S[j - 1];
                    float qbbm = 0.f;
                    if (ty != 0) {
                        float a_int = 0.f;
                        const float *pp = L.part + (pe * 2 + fl) * OX_NB * WAVE + lane;
#pragma unroll
                        for (int b = 0; b < OX_NB; b++) a_int += pp[b * WAVE];
                        const float ext = L.dt[DT_EXT + ty * 36 + ((i > 1) ? S[i - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
                        const float stem = L.dt[DT_MLS + ty * 25 + S[i - 1] * 5 + S[j + 1]];
                        const float qbb = a_int + L.q5b[j] * L.q5[i - 1] * ext + qm1b * stem;
                        qbbm = qbb * L.dt[DT_MMI + oc];
                        if (e - 2 >= 4)   // X(i+1, j-1): this pair closing a multiloop
                            L.Y[off(e - 2, N) + i] =
                                qbb * mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
                        if (motif && e == mL - 1 && L.mat[i])
                            L.pm[i] = float(double(qbb) * XS->motif_extra / Z);
                        for (int t = 0; t < ka.n_pairs && t < OX_MAXP; t++) {
                            if (ka.pairs[3 * t] == bv && ka.pairs[3 * t + 1] == i && ka.pairs[3 * t + 2] == j) {
                                const int cc = rtype(ty) * 25 + S[j + 1] * 5 + S[i - 1];
                                const double qb = double(src[ce]) * double(ct[CT_INVMM + cc]);
                                L.pd[t] = qb * double(qbb) / double(Z);
                            }
                        }
                    }
                    const int wo = wslot(e) * L.RL + OX_PAD + i - 1;
                    L.qw[wo] = qbbm;
                    L.ow[wo] = uint8_t(oc);
                }
            }
        }
        lds_barrier();
    }
    // ---- requested pairs of this fold (score terms), the motif's inner pairs credited
    // from its closing cell (kernels.hip outside())
    double *pp = pair_p + size_t(w) * ka.n_pairs;
    for (int t = tid; t < ka.n_pairs; t += OX_NT) {
        if (ka.pairs[3 * t] != bv) continue;
        const int i = ka.pairs[3 * t + 1], j = ka.pairs[3 * t + 2];
        double pij = 0.0;
        if (i >= 1 && j <= N && j - i >= 4) {
            pij = t < OX_MAXP ? L.pd[t] : 0.0;
            if (motif)
                for (int o = 1; o + mL - 1 <= N; o++) {
                    if (o + mL - 1 < j || i < o) continue;
                    const float pmo = L.pm[o];
                    if (pmo == 0.f) continue;
                    const int pk = XS->motif_pt[i - o];
                    if (i - o >= 1 && pk == j - o) pij += pmo;
                }
        }
        pp[t] = pij;
    }
}

}  // namespace

// LDS bytes of the lanes = cells outside kernel for this workload (0: not covered)
size_t outside_cells_lds(const KArgs &ka) {
    if (ka.Nmax > OX_NMAX || ka.Nmax < 8 || ka.n_pairs > OX_MAXP || !ka.tab) return 0;
    const size_t b = OxLay(ka.Nmax).BYTES;
    return b + 256 <= 160 * 1024 ? b : 0;
}

hipError_t launch_outside_cells(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *pair_p,
                                int sp_score, hipStream_t stream) {
    const size_t lds = outside_cells_lds(ka);
    if (lds == 0) return hipErrorInvalidValue;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(outside_cells_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(outside_cells_kernel, dim3(W * ka.n_bvars), dim3(OX_NT), lds, stream, ka, ka.X, seqs, W, mask,
                       pair_p, sp_score);
    return hipGetLastError();
}

}  // namespace adx
