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
//     over 10 waves (B); waves 10-15 sum the multiloop adjoints (M) over row- /
//     column-major copies of Y, qm1 and qm (consecutive rows / columns of a
//     triangular table start in distinct banks, so a split point is one
//     conflict-free read per lane at an immediate offset); the next step
//     finalizes the cell (F).
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
// unconstrained folds, adx_api.cpp), N <= 112 (LDS); everything else takes
// kernels.hip bppm_kernel.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "dev_types.hpp"
#include "fold_common.hpp"

#ifndef MS_CH
#define MS_CH 4   // terms per multiloop-sum read step (even; 16: 423k, 4: 430k, 2: 424k config-3 MC steps/s)
#endif

namespace adx {

#ifdef ADX_STAMP
// Diagnostic build only: per-wave cycle sums of the phases (s_memtime), read
// back through adx_debug_stamps_outside().  Never in the product.
__device__ unsigned long long g_stamps_o[16][8];
#define OSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define OSTAMP(k) do { } while (0)
#endif
}  // namespace adx

#include "outside_common.hpp"

namespace adx {

namespace {

constexpr int OX_NMAX = 112;
#ifndef OX_PART
#define OX_PART 0   // interior-loop size partition of the B waves (A/B knob)
#endif
constexpr int OX_SLACK = 64;          // zeroed floats after each cell table (reads past a row end)

// LDS carve for folded length N (runtime; the host sizes the launch with it)
struct OxLay {
    int C, NP, RL;
    size_t YR, YC, Q1R, QMC, QW, OW, PART, MLP, REC, CL, FR, SF, RQ, RR, R1, Q5, Q5B, PM, CT, DT, PD, PL, S, MT, BYTES;
    __host__ __device__ static size_t a16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ explicit OxLay(int N) {
        C = ((N - 4) * (N - 3)) / 2;
        NP = N + 2;
        RL = N + 2 * OX_PAD;
        size_t o = 0;
        const size_t T = a16((size_t(C) + OX_SLACK) * 4);
        YR = o;   o += T;                                        // Y row-major (qmb sums)
        YC = o;   o += T;                                        // Y column-major (r2 sums; G before the sweep)
        Q1R = o;  o += T;                                        // inside qm1, row-major
        QMC = o;  o += T;                                        // inside qm, column-major
        QW = o;   o += a16(size_t(OX_WIN) * RL * 4);             // qbb * mismatchI(outer) window
        OW = o;   o += a16(size_t(OX_WIN) * RL);                 // outer codes window
        PART = o; o += a16(size_t(2) * 2 * OX_NB * WAVE * 4);   // [parity][lane-set][block][lane]
        MLP = o;  o += a16(size_t(2) * OX_NM * WAVE * 4);       // [parity][M wave][lane]
        REC = o;  o += a16(size_t(2) * 2 * OX_RF * WAVE * 4 + 16);   // cell setup records [parity][lane-set][field][lane]; counts [parity]
        CL = o;   o += a16(size_t(C) + size_t(NP));              // pairable cells per diagonal: cl[off(D) + rank] = i; counts
        FR = o;   o += a16(size_t(2) * 2 * OX_FF * WAVE * 4);   // finalize records [parity][lane-set][field][lane]
        SF = o;   o += a16(size_t(31) * 32 * 4);                 // constant factor of shape (u, n1): [u][n1]
        RQ = o;   o += a16(size_t(2) * NP * 4);                  // qmb ring [parity][i]
        RR = o;   o += a16(size_t(2) * NP * 4);                  // R ring
        R1 = o;   o += a16(size_t(2) * NP * 4);                  // qm1b ring
        Q5 = o;   o += a16(size_t(NP) * 4);
        Q5B = o;  o += a16(size_t(NP) * 4);
        PM = o;   o += a16(size_t(NP) * 4);                      // motif site weights
        CT = o;   o += a16(size_t(CT_SIZE) * 4);
        DT = o;   o += a16(size_t(DT_EXT + 288) * 4);            // MMI, MLS, EXT
        PD = o;   o += a16(size_t(OX_MAXP) * 8);                 // requested pairs: qb qbb / Z
        PL = o;   o += a16(size_t(OX_MAXP) * 4 + 4);             // this fold's pairs: t | i << 8 | j << 16; count
        S = o;    o += a16(size_t(NP) + 8);
        MT = o;   o += a16(size_t(NP));                          // motif site flags
        BYTES = o;
    }
};

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
    L.yr = reinterpret_cast<float *>(smem + Y.YR);
    L.yc = reinterpret_cast<float *>(smem + Y.YC);
    L.q1r = reinterpret_cast<float *>(smem + Y.Q1R);
    L.qmc = reinterpret_cast<float *>(smem + Y.QMC);
    L.pl = reinterpret_cast<int *>(smem + Y.PL);
    L.qw = reinterpret_cast<float *>(smem + Y.QW);
    L.ow = reinterpret_cast<uint8_t *>(smem + Y.OW);
    L.part = reinterpret_cast<float *>(smem + Y.PART);
    L.mlp = reinterpret_cast<float *>(smem + Y.MLP);
    L.rec = reinterpret_cast<float *>(smem + Y.REC);
    L.rcnt = reinterpret_cast<int *>(smem + Y.REC + size_t(2) * 2 * OX_RF * WAVE * 4);
    L.cl = reinterpret_cast<uint8_t *>(smem + Y.CL);
    uint8_t *cn = L.cl + Y.C;   // cn[D]: pairable cells of diagonal D
    L.sf = reinterpret_cast<float *>(smem + Y.SF);
    L.fr = reinterpret_cast<float *>(smem + Y.FR);
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
    // physical wave -> role: the finalize roles (0, 1) run on waves 2, 3 and the
    // finalize-record roles (2, 3) on waves 0, 1, so the finalize shares its SIMDs
    // with fewer multiloop-sum waves (config 3 462.5k -> 470.3k MC steps/s,
    // profiles/r04zd_ab_wperm.txt; OX_WPERM overrides it in diagnostic builds)
#ifndef OX_WPERM
#define OX_WPERM 2, 3, 0, 1, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15
#endif
    constexpr int wperm[OX_NW] = {OX_WPERM};
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(wperm[tid / WAVE]);
    const int C = Y.C, NP = Y.NP;
#ifdef ADX_STAMP
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    const DevTables &T = *ka.T;

    // ---- the proposal's inside tables (score_kernel's P = sp_score layout, kernels.hip Inc)
    const size_t B = 3 * size_t(ka.cells) + size_t(ka.Nmax) + 2;
    const size_t go = (sp_score == 2 ? size_t(ka.bvar_slot[bv]) : size_t(v)) * B;
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
    // constant factor of each shape (u, n1): generic fgen, bulge / 1xn length
    // factors, the sigma powers of the tabulated loops (adx_api.cpp addS)
    for (int k = tid; k < 31 * 32; k += OX_NT) {
        const int u = k >> 5, n1 = k & 31, n2 = u - n1;
        float f = 0.f;
        if (n1 <= u) {
            const int kd = okind(n1, n2);
            f = kd < 0 ? XS->fgen[(u - 6) * FG_ROW + n1 - 2]
              : kd == TK_STK ? XS->ctab[CT_FSM + 0]
              : kd == TK_B1 ? XS->ctab[CT_FSM + 1]
              : kd == TK_BUL ? XS->ctab[CT_FB + u]
              : kd == TK_1N ? XS->ctab[CT_F1N + u - 1]
              : kd == TK_I11 ? XS->ctab[CT_FSM + 2]
              : kd == TK_I22 ? XS->ctab[CT_FSM + 4]
              : kd == TK_M23 ? XS->ctab[CT_FSM + 5]
              : XS->ctab[CT_FSM + 3];   // 1x2 / 2x1
        }
        L.sf[k] = f;
    }
    for (int k = tid; k <= N; k += OX_NT) L.q5[k] = src[3 * Cs + k];
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

    // this fold's requested pairs (score terms), kept in LDS for the finalize
    if (tid == 0) {
        int n = 0;
        for (int t = 0; t < ka.n_pairs && t < OX_MAXP; t++)
            if (ka.pairs[3 * t] == bv) L.pl[n++] = t | (ka.pairs[3 * t + 1] << 8) | (ka.pairs[3 * t + 2] << 16);
        L.pl[OX_MAXP] = n;
    }
    // inside tables, one flat pass over the cells: qm1 row-major and qm
    // column-major (transposed from the slot's column- / row-major), Y row-major
    // zeroed; the exterior factors G(i, j) = qb(i,j) ext(i,j) column-major in the
    // YC region (zeroed after the exterior adjoint)
    float *G = L.yc;
#pragma unroll 2
    for (int k = tid; k < C + OX_SLACK; k += OX_NT) {
        if (k >= C) {   // slack after each table: finite zeros for reads past a row end
            L.yr[k] = L.q1r[k] = L.qmc[k] = G[k] = 0.f;
            continue;
        }
        const int i = inv_off(k, N) - 3, l = i + 4 + (k - rowb(i, N));   // row-major cell (i, l): rowb == off(i + 3)
        L.q1r[k] = src[2 * Cs + colb(l) + i - 1];
        L.yr[k] = 0.f;
        const int jc = inv_colb(k), ic = k - colb(jc) + 1;                 // column-major cell (ic, jc)
        L.qmc[k] = src[Cs + rowb(ic, N) + jc - ic - 4];
        const int ty = ptype(S[ic], S[jc]);
        const int cc = rtype(ty) * 25 + S[jc + 1] * 5 + S[ic - 1];
        const float e = L.dt[DT_EXT + ty * 36 + ((ic > 1) ? S[ic - 1] : 5) * 6 + ((jc < N) ? S[jc + 1] : 5)];
        G[k] = src[off(jc - ic, N) + ic - 1] * (ct[CT_INVMM + cc] * e);   // non-pairable: -0 * x = 0
    }
    __syncthreads();

    OSTAMP(0);   // loads + table pass
    // ---- exterior adjoint (kernels.hip outside(), push form, one wave, lanes = m):
    // once q5b[j] is known every m <= j-5 takes q5b[j] G(m+1, j).  acc[j-5] is
    // final after the push of j, and q5b[j-5] needs it four steps later, so the
    // loop-carried chain is one FMA: q5b[j-1] = sigma q5b[j] + acc[j-1], acc[j-1]
    // read (readlane) four iterations ahead; the next column of G is loaded
    // during the current push.
    if (wid == 0) {
        const float sig1 = XS->sig[1];
        float acc0 = 0.f, acc1 = 0.f;   // m = lane, m = 64 + lane
        float val = 1.f;                // q5b[N]
        float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;   // acc[j-1], acc[j-2], acc[j-3], acc[j-4]
        if (lane == 0) L.q5b[N] = 1.f;
        float g0 = 0.f, g1 = 0.f;       // G column j for lanes m, 64 + m
        if (N >= 5) {
            const int cb = colb(N);
            g0 = G[cb + min(lane, N - 5)];
            g1 = G[cb + min(WAVE + lane, N - 5)];
        }
        for (int j = N; j >= 1; j--) {
            float n0 = 0.f, n1 = 0.f;   // prefetch: column j - 1
            if (j - 1 >= 5) {
                const int cb = colb(j - 1);
                n0 = G[cb + min(lane, j - 6)];
                n1 = G[cb + min(WAVE + lane, j - 6)];
            }
            if (j >= 5) {
                if (lane <= j - 5) acc0 = fmaf(val, g0, acc0);
                if (WAVE + lane <= j - 5) acc1 = fmaf(val, g1, acc1);
            }
            // acc[j-5] is final now
            const int m5 = j - 5;
            float a5 = 0.f;
            if (m5 >= 0)
                a5 = __int_as_float(m5 < WAVE ? __builtin_amdgcn_readlane(__float_as_int(acc0), m5)
                                              : __builtin_amdgcn_readlane(__float_as_int(acc1), m5 - WAVE));
            val = fmaf(sig1, val, q0);   // q5b[j-1]
            if (lane == 0) L.q5b[j - 1] = val;
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = a5;
            g0 = n0;
            g1 = n1;
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
    // while wave 0 runs the exterior adjoint: the window zeroed and the pairable
    // cells of every diagonal in rank order (the B lanes; an unconstrained fold:
    // the pair type alone decides), on waves 2.. (neither touches G)
    if (wid >= 2) {
        const int t2 = (wid - 2) * WAVE + lane, n2 = OX_NT - 2 * WAVE;
        for (int k = t2; k < OX_WIN * L.RL; k += n2) {
            L.qw[k] = 0.f;
            L.ow[k] = 0;
        }
        for (int D = 4 + wid - 2; D <= N - 1; D += OX_NW - 2) {
            const int od = off(D, N);
            int base = 0;
            for (int i0 = 1; i0 <= N - D; i0 += WAVE) {
                const int i = i0 + lane;
                const bool pr = i <= N - D && ptype(S[i], S[i + D]) != 0;
                const uint64_t m = __ballot(pr);
                const int slot = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                if (pr) L.cl[od + slot] = uint8_t(i);
                base += __popcll(m);
            }
            if (lane == 0) cn[D] = uint8_t(base);
        }
    }
    __syncthreads();
    for (int k = tid; k < C; k += OX_NT) L.yc[k] = 0.f;   // G's region: Y column-major from here on
    __syncthreads();

    OSTAMP(1);   // exterior adjoint + zeroing
    const float mlbase_sig = XS->mlbase_sig, mlclosing = XS->mlclosing, pw1 = XS->pwml[1];

    // Setup record of the cells of lane-set ls of diagonal D, written one step
    // before B reads it: inner mismatch, TermAU, 1xn / 2x3 factors of the cell as
    // the inner pair, the four 1x1..2x2 table factors (loaded from HBM one more
    // step ahead, tab_load), type | pairable.
    auto cell_of = [&](int D, int ls, int &i, int &j) {
        i = 1 + ls * WAVE + lane;
        const bool valid = i <= N - D;
        if (!valid) i = N - D;
        j = i + D;
        return valid;
    };
    // The records of diagonal D's pairable cells (rank lists built in setup) in
    // three stages a step apart, one LDS round trip each: idx_load (rank list),
    // tab_load (bases, the cell's LDS factors, the 1x1..2x2 table factors from
    // HBM/L2), rec_write (stores only).
    struct Idx {
        int cnt;
        int i[2];   // the lane's cell (cell 1 on idle lanes: its shapes are read and discarded)
    };
    auto idx_load = [&](int D) {
        Idx X;
        X.cnt = 0;
        X.i[0] = X.i[1] = 1;
        if (D < 4) return X;
        const int od = off(D, N);
        X.cnt = uni(cn[D]);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int idx = k * WAVE + lane;
            const int ir = L.cl[od + min(idx, N - D - 1)];
            X.i[k] = idx < X.cnt ? ir : 1;
        }
        return X;
    };
    struct Pend {
        int cnt;
        int i[2], ty2[2];
        float mmin[2], mo[2], m23[2];
        float4 t[2];
    };
    auto tab_load = [&](int D, const Idx &X) {
        Pend P;
        P.cnt = X.cnt;
        const int umax = min(30, N - 3 - D);
        auto Sc = [&](int x) { return int(S[x < 0 ? 0 : (x > N + 1 ? N + 1 : x)]); };
#pragma unroll
        for (int k = 0; k < 2; k++) {
            P.i[k] = X.i[k];
            P.ty2[k] = 0;
            P.mmin[k] = P.mo[k] = P.m23[k] = 0.f;
            P.t[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (k * WAVE >= X.cnt) continue;
            const int i = X.i[k], j = i + D;
            const int ty2 = rtype(ptype(S[i], S[j]));
            const int cc = ty2 * 25 + S[j + 1] * 5 + S[i - 1];
            P.ty2[k] = ty2;
            P.mmin[k] = L.dt[DT_MMI + cc];
            P.mo[k] = ct[CT_ONEN + cc] * P.mmin[k];
            P.m23[k] = ct[CT_M23O + cc];
            float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
            if (umax >= 2) t.x = T.int11[ptype(Sc(i - 2), Sc(j + 2))][ty2][Sc(i - 1)][Sc(j + 1)];
            if (umax >= 3) {
                t.y = T.int21[ptype(Sc(i - 2), Sc(j + 3))][ty2][Sc(i - 1)][Sc(j + 1)][Sc(j + 2)];
                t.z = T.int21[ty2][ptype(Sc(i - 3), Sc(j + 2))][Sc(j + 1)][Sc(i - 2)][Sc(i - 1)];
            }
            if (umax >= 4) t.w = T.int22[ptype(Sc(i - 3), Sc(j + 3))][ty2][Sc(i - 2)][Sc(i - 1)][Sc(j + 1)][Sc(j + 2)];
            P.t[k] = t;
        }
        return P;
    };
    // records of diagonal D's compacted pairable cells (read by B at step D)
    auto rec_write = [&](int D, const Pend &P) {
        if (D < 4) return;
        if (lane == 0) L.rcnt[D & 1] = P.cnt;
        for (int k = 0; k < 2; k++) {
            const int idx = k * WAVE + lane;
            if (k * WAVE >= P.cnt) break;
            const bool v = idx < P.cnt;
            float *r = L.rec + (((D & 1) * 2 + k) * OX_RF) * WAVE + lane;
            // an idle lane reads cell 1's shapes (discarded)
            r[0 * WAVE] = __int_as_float(P.i[k] | (P.ty2[k] << 8) | (v ? (1 << 16) : 0));
            r[1 * WAVE] = P.mmin[k];
            r[2 * WAVE] = P.mo[k];
            r[3 * WAVE] = P.m23[k];
            r[4 * WAVE] = P.t[k].x;
            r[5 * WAVE] = P.t[k].y;
            r[6 * WAVE] = P.t[k].z;
            r[7 * WAVE] = P.t[k].w;
        }
    };
    constexpr int RW = 7;   // B wave RW: setup records (both lane-sets)
    Pend pnext;             // the factors of the diagonal after the next
    Idx inext;              // the rank list of the one after that
    pnext.cnt = 0;
    inext.cnt = 0;
    if (wid == RW) {
        rec_write(N - 1, tab_load(N - 1, idx_load(N - 1)));
        pnext = tab_load(N - 2, idx_load(N - 2));
        inext = idx_load(N - 3);
    }
    __syncthreads();

    // Finalize record of lane-set ls of diagonal e (written at step e, read by F
    // at step e - 1): the cell's exterior term q5b[j] q5[i-1] ext, multiloop stem,
    // outer mismatch, multiloop-closing factor of the pair, type | code | pairable.
    auto frec_write = [&](int e, int ls) {
        if (e < 4 || ls >= (N - e + WAVE - 1) / WAVE) return;
        int i, j;
        const bool valid = cell_of(e, ls, i, j);
        const int ty = ptype(S[i], S[j]);
        const int oc = ty * 25 + S[i + 1] * 5 + S[j - 1];
        float *r = L.fr + (((e & 1) * 2 + ls) * OX_FF) * WAVE + lane;
        r[0] = L.q5b[j] * L.q5[i - 1] * L.dt[DT_EXT + ty * 36 + ((i > 1) ? S[i - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
        r[WAVE] = L.dt[DT_MLS + ty * 25 + S[i - 1] * 5 + S[j + 1]];
        r[2 * WAVE] = L.dt[DT_MMI + oc];
        r[3 * WAVE] = mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
        r[4 * WAVE] = __int_as_float(ty | (oc << 8) | ((valid && ty != 0) ? (1 << 16) : 0));
    };

    // ---------------- F: finalize diagonal e = d + 1, lane-set fl (after the
    // step's B work, on B waves 0 and 1): one batch of independent reads
    auto finalize = [&](int d, int fl) {
        const int e = d + 1;
        const int nle = (N - e + WAVE - 1) / WAVE;
        if (e > N - 1 || fl >= nle) return;
        const int pe = e & 1, pn = (e + 1) & 1;
        const int i = 1 + fl * WAVE + lane;
        if (i > N - e) return;
        const int j = i + e;
        const bool te = nle == 2;
        const float *mp = L.mlp + pe * OX_NM * WAVE + lane;
        const float qmbv = te ? (fl ? mp[2 * WAVE] : mp[0] + mp[WAVE]) : mp[0] + mp[WAVE] + mp[2 * WAVE];
        const float r2 = te ? (fl ? mp[4 * WAVE] + mp[5 * WAVE] : mp[3 * WAVE]) : mp[3 * WAVE] + mp[4 * WAVE] + mp[5 * WAVE];
        const float R = i >= 2 ? pw1 * (L.rq[pn * NP + i - 1] + L.rr[pn * NP + i - 1]) : 0.f;
        const float chain = j < N ? mlbase_sig * L.r1[pn * NP + i] : 0.f;
        const float qm1b = qmbv + R + r2 + chain;
        const float *fr = L.fr + ((pe * 2 + fl) * OX_FF) * WAVE + lane;
        const int tp = __float_as_int(fr[4 * WAVE]);
        float a_int = 0.f;   // B wrote the partials of every pairable cell when an outer loop fits
        const float *pp = L.part + (pe * 2 + fl) * OX_NB * WAVE + lane;
#pragma unroll
        for (int b = 0; b < OX_NB; b++) a_int += pp[b * WAVE];
        if (N - 3 - e < 0) a_int = 0.f;
        L.rq[pe * NP + i] = qmbv;
        L.rr[pe * NP + i] = R;
        L.r1[pe * NP + i] = qm1b;
        L.yr[rowb(i, N) + e - 4] += qmbv;   // Y(i, j): X(i, j) was stored two diagonals ago
        L.yc[colb(j) + i - 1] += qmbv;
        float qbbm = 0.f;
        if (tp >> 16) {
            const float qbb = a_int + fr[0] + qm1b * fr[WAVE];
            qbbm = qbb * fr[2 * WAVE];
            if (e - 2 >= 4) {   // X(i+1, j-1): this pair closing a multiloop
                const float x = qbb * fr[3 * WAVE];
                L.yr[rowb(i + 1, N) + e - 6] = x;
                L.yc[colb(j - 1) + i] = x;
            }
            if (motif && e == mL - 1 && L.mat[i]) L.pm[i] = float(double(qbb) * XS->motif_extra / Z);
            const int npl = L.pl[OX_MAXP];
            for (int q = 0; q < npl; q++) {
                const int pk = L.pl[q];
                if (((pk >> 8) & 255) == i && (pk >> 16) == j) {
                    const int cc = rtype(tp & 255) * 25 + S[j + 1] * 5 + S[i - 1];
                    const double qb = double(src[off(e, N) + i - 1]) * double(ct[CT_INVMM + cc]);
                    L.pd[pk & 255] = qb * double(qbb) / double(Z);
                }
            }
        }
        const int wo = wslot(e) * L.RL + OX_PAD + i - 1;
        L.qw[wo] = qbbm;
        L.ow[wo] = uint8_t((tp >> 8) & 255);
    };
    auto fin = [&](int d, auto wc) {
        constexpr int w = decltype(wc)::value;
        if constexpr (w < 2) {
            finalize(d, w);
        } else if constexpr (w < 4) {
            frec_write(d, w - 2);   // diagonal d, finalized next step
        } else if (w == RW) {
            // setup records of diagonal d - 1 (next step's B) from the factors made last
            // step; the factors of diagonal d - 2, the rank list of d - 3
            rec_write(d - 1, pnext);
            pnext = tab_load(d - 2, inext);
            inext = idx_load(d - 3);
        }
    };

    // ---- the sweep: step d runs B and M of diagonal d and F of diagonal d + 1.
    // B: loop sizes in blocks of about equal cost (generic shape ~2 instructions,
    // a special ~9); the 1x1..2x2 table shapes (u = 2, 3, 4) last in their blocks
    if (wid < OX_NB) {
        switch (wid) {
            // loop sizes spread so that every wave's B blocks plus its other role take
            // about the same time (stamps, tools/outside_stamps.py): the finalize
            // wave 0 one size and the record wave 7 none (a size >= 6 costs 3 reads for its
            // special shapes + one per 4 generic ones per lane-set, sizes <= 5 ~3 per shape)
            case 0: b_sweep<2, 19, -1, -1, -1, -1>(L, N, lane, std::integral_constant<int, 0>{}, fin OX_STP_ARGS); break;
            case 1: b_sweep<2, 5, 7, 15, -1, -1>(L, N, lane, std::integral_constant<int, 1>{}, fin OX_STP_ARGS); break;
            case 2: b_sweep<2, 4, 0, 23, -1, -1>(L, N, lane, std::integral_constant<int, 2>{}, fin OX_STP_ARGS); break;
            case 3: b_sweep<2, 3, 30, 6, 11, -1>(L, N, lane, std::integral_constant<int, 3>{}, fin OX_STP_ARGS); break;
            case 4: b_sweep<2, 29, 28, 27, 1, -1>(L, N, lane, std::integral_constant<int, 4>{}, fin OX_STP_ARGS); break;
            case 5: b_sweep<2, 26, 25, 24, 2, -1>(L, N, lane, std::integral_constant<int, 5>{}, fin OX_STP_ARGS); break;
#if OX_PART == 1   // (A/B knobs) size 10 from block 8 to the record wave 7, size 9 from block 9 to block 6
            case 6: b_sweep<2, 22, 21, 20, 8, 9>(L, N, lane, std::integral_constant<int, 6>{}, fin OX_STP_ARGS); break;
            case 7: b_sweep<2, 10, -1, -1, -1, -1>(L, N, lane, std::integral_constant<int, 7>{}, fin OX_STP_ARGS); break;
            case 8: b_sweep<2, 18, 17, 16, -1, -1>(L, N, lane, std::integral_constant<int, 8>{}, fin OX_STP_ARGS); break;
            default: b_sweep<2, 14, 13, 12, -1, -1>(L, N, lane, std::integral_constant<int, 9>{}, fin OX_STP_ARGS); break;   // wave 9
#elif OX_PART == 2   // size 10 from block 8 to the record wave 7
            case 6: b_sweep<2, 22, 21, 20, 8, -1>(L, N, lane, std::integral_constant<int, 6>{}, fin OX_STP_ARGS); break;
            case 7: b_sweep<2, 10, -1, -1, -1, -1>(L, N, lane, std::integral_constant<int, 7>{}, fin OX_STP_ARGS); break;
            case 8: b_sweep<2, 18, 17, 16, -1, -1>(L, N, lane, std::integral_constant<int, 8>{}, fin OX_STP_ARGS); break;
            default: b_sweep<2, 14, 13, 12, 9, -1>(L, N, lane, std::integral_constant<int, 9>{}, fin OX_STP_ARGS); break;   // wave 9
#elif OX_PART == 3   // size 10 from block 8 to block 6
            case 6: b_sweep<2, 22, 21, 20, 8, 10>(L, N, lane, std::integral_constant<int, 6>{}, fin OX_STP_ARGS); break;
            case 7: b_sweep<2, -1, -1, -1, -1, -1>(L, N, lane, std::integral_constant<int, 7>{}, fin OX_STP_ARGS); break;
            case 8: b_sweep<2, 18, 17, 16, -1, -1>(L, N, lane, std::integral_constant<int, 8>{}, fin OX_STP_ARGS); break;
            default: b_sweep<2, 14, 13, 12, 9, -1>(L, N, lane, std::integral_constant<int, 9>{}, fin OX_STP_ARGS); break;   // wave 9
#else
            case 6: b_sweep<2, 22, 21, 20, 8, -1>(L, N, lane, std::integral_constant<int, 6>{}, fin OX_STP_ARGS); break;
            case 7: b_sweep<2, -1, -1, -1, -1, -1>(L, N, lane, std::integral_constant<int, 7>{}, fin OX_STP_ARGS); break;
            case 8: b_sweep<2, 18, 17, 16, 10, -1>(L, N, lane, std::integral_constant<int, 8>{}, fin OX_STP_ARGS); break;
            default: b_sweep<2, 14, 13, 12, 9, -1>(L, N, lane, std::integral_constant<int, 9>{}, fin OX_STP_ARGS); break;   // wave 9
#endif
        }
    } else for (int d = N - 1; d >= 3; d--) {
        const int nls = d >= 4 ? (N - d + WAVE - 1) / WAVE : 0;   // lane-sets of diagonal d
        const int par = d & 1;
        {
            // ---------------- M: multiloop adjoint sums of diagonal d.  Work items:
            // two lane-sets: qmb ls0 (halves on waves 0, 1), qmb ls1, r2 ls0, r2 ls1
            // (halves on 4, 5); one lane-set: qmb and r2 in thirds
            const int mw = wid - OX_NB;
            if (d >= 4) {
                const bool two = nls == 2;
                const bool isq = mw < 3;
                const int ls = two ? ((mw == 2 || mw >= 4) ? 1 : 0) : 0;
                const int np = two ? ((mw <= 1 || mw >= 4) ? 2 : 1) : 3;                 // parts of the item
                const int pi = two ? (mw == 1 || mw == 5 ? 1 : 0) : (mw % 3);            // this wave's part
                int i = 1 + ls * WAVE + lane;
                const int ilast = min(N - d, (ls + 1) * WAVE);
                const bool valid = i <= N - d;
                if (!valid) i = N - d;
                const int j = i + d;
                float acc = 0.f, acc1 = 0.f;
                // sum_t y[t] q[t] over t = ta .. tl (the lane's own bound), MS_CH terms
                // per step: the loop ends at the lane's range, so a lane reads at most
                // MS_CH - 1 terms past it (each a wasted LDS cycle on the chain the
                // step waits on; pf_cells.hip qm items); even offsets into acc, odd
                // into acc1, in order -- bit-identical to the 16-wide chunks
                auto msum = [&](const float *py, const float *pq, int ta, int tl, float &a0, float &a1) {
                    for (int t = ta; t <= tl; t += MS_CH) {
                        float yv[MS_CH], qv[MS_CH];
#pragma unroll
                        for (int k = 0; k < MS_CH; k++) { yv[k] = py[t + k]; qv[k] = pq[t + k]; }
#pragma unroll
                        for (int k = 0; k < MS_CH; k += 2) {
                            a0 = fmaf(t + k <= tl ? yv[k] : 0.f, qv[k], a0);
                            a1 = fmaf(t + k + 1 <= tl ? yv[k + 1] : 0.f, qv[k + 1], a1);
                        }
                    }
                };
                if (isq) {
                    // qmb: t = 0 .. N-j-5: Y(i, j+5+t) = YR[rowb(i) + d + 1 + t],
                    // qm1(j+1, j+5+t) = Q1R[rowb(j+1) + t]
                    const int lim = N - j - 5;
                    const int T = N - (1 + ls * WAVE + d) - 4;          // the lane-set's longest range
                    const int ta = (T * pi) / np, tb = (T * (pi + 1)) / np;
                    const float *py = L.yr + rowb(i, N) + d + 1, *pq = L.q1r + rowb(j + 1, N);
                    msum(py, pq, ta, min(lim, tb - 1), acc, acc1);
                } else {
                    // r2: ip = 1 .. i-5: Y(ip, j) = YC[colb(j) + ip - 1], qm(ip, i-1) = QMC[colb(i-1) + ip - 1]
                    const int lim = i - 5;
                    const int T = ilast - 5;
                    const int ta = 1 + (T * pi) / np, tb = 1 + (T * (pi + 1)) / np;
                    const float *py = L.yc + colb(j) - 1, *pq = L.qmc + colb(i - 1) - 1;
                    msum(py, pq, ta, min(lim, tb - 1), acc, acc1);
                }
                L.mlp[(par * OX_NM + mw) * WAVE + lane] = acc + acc1;
            }
            OSTAMP(4);   // M sums
        }
        OSTAMP(5);   // F (M waves) / B tail
        lds_barrier();
        OSTAMP(6);   // barrier
    }
#ifdef ADX_STAMP
    if (lane == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_stamps_o[wid][k], st_acc[k]);
#endif
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
    const OxLay y(ka.Nmax);
    return y.BYTES + 256 <= 160 * 1024 ? y.BYTES : 0;
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

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_outside(unsigned long long *out, int reset) {  // [16][8]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_o), sizeof(adx::g_stamps_o)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_o), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
