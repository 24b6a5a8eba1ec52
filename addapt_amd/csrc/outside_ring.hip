// gfx950 outside pass (base-pair probabilities, BASELINE config 4: N = 150)
// with lanes = cells, for the folds pf_ring_kernel (pf_ring.hip) leaves in the
// walker's table slot -- the equations of outside_cells.hip (the adjoint of the
// inside recursions in gather form, descending span order), with the LDS
// carved for lengths where outside_cells' four cell tables (4 x 43 KB at
// N = 150) do not fit:
//
//   * Y = qmb + X stays in LDS, ROW-major only (43 KB).  The r2 sum walks a
//     column of Y: lane (i, j) reads Y(i-u, j) at rowb(i-u) + d + u - 4, a
//     per-lane base that moves by an add per term (consecutive rows start in
//     distinct banks, so the reads stay conflict-free);
//   * the inside tables qm1 and qm are read from the slot, where pf_ring_kernel
//     keeps them DIAGONAL-major: with lanes = consecutive cells, the term
//     qm1(j+1, j+5+t) of every lane lies on diagonal t+4 and qm(i-u, i-1) on
//     diagonal u-1, so each term is one coalesced global load (L2-resident:
//     86 KB per fold);
//   * three lane-sets per diagonal (N - 4 <= 192): three finalize waves, three
//     record sets, the multiloop items one per M wave.
//
// Covered: pf_ring contexts (unconstrained folds with pair terms, N <= the
// LDS limit); kernels.hip chooses it with the inside kernel.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {
#ifdef ADX_STAMP
// Diagnostic build only: per-wave cycle sums of the phases (s_memtime), read
// back through adx_debug_stamps_outside_ring().  Never in the product.
__device__ unsigned long long g_stamps_or[16][8];
#define OSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#endif
}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_outside_ring(unsigned long long *out, int reset) {  // [16][8]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_or), sizeof(adx::g_stamps_or)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_or), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif

#include "outside_common.hpp"

namespace adx {
namespace {

constexpr int OR_SETS = 3;
constexpr int OR_NB = 8;              // interior-loop waves 0-7 (records on 7); multiloop sums on 8-15
constexpr int OR_NMIN = 101, OR_NMAX = 190;
constexpr int OR_SLACK = 64;

struct OrLay {
    int C, NP, RL;
    size_t YR, QW, OW, PART, MLP, REC, CL, FR, SF, RQ, RR, R1, Q5, Q5B, PM, CT, DT, PD, PL, S, MT, BYTES;
    __host__ __device__ static size_t a16(size_t b) { return (b + 15) & ~size_t(15); }
    __host__ __device__ explicit OrLay(int N) {
        C = ((N - 4) * (N - 3)) / 2;
        NP = N + 2;
        RL = ((N + OX_PAD + 4) + 3) & ~3;   // window row: outer a from i-31 (zero pad in front)
        size_t o = 0;
        YR = o;   o += a16((size_t(C) + OR_SLACK) * 4);          // Y row-major (G column-major before the sweep)
        QW = o;   o += a16(size_t(OX_WIN) * RL * 4);             // qbb * mismatchI(outer) window
        OW = o;   o += a16(size_t(OX_WIN) * RL);                 // outer codes window
        PART = o; o += a16(size_t(2) * OR_SETS * OX_NB * WAVE * 4);
        MLP = o;  o += a16(size_t(2) * OX_NW * WAVE * 4);           // M parts: [parity][wave][lane]
        REC = o;  o += a16(size_t(2) * OR_SETS * OX_RF * WAVE * 4 + 16);
        CL = o;   o += a16(size_t(C) + size_t(NP));
        FR = o;   o += a16(size_t(2) * OR_SETS * OX_FF * WAVE * 4);
        SF = o;   o += a16(size_t(31) * 32 * 4);
        RQ = o;   o += a16(size_t(2) * NP * 4);
        RR = o;   o += a16(size_t(2) * NP * 4);
        R1 = o;   o += a16(size_t(2) * NP * 4);
        Q5 = o;   o += a16(size_t(NP) * 4);
        Q5B = o;  o += a16(size_t(NP) * 4);
        PM = o;   o += a16(size_t(NP) * 4);
        CT = o;   o += a16(size_t(CT_SIZE) * 4);
        DT = o;   o += a16(size_t(DT_EXT + 288) * 4);
        PD = o;   o += a16(size_t(OX_MAXP) * 8);
        PL = o;   o += a16(size_t(OX_MAXP) * 4 + 4);
        S = o;    o += a16(size_t(NP) + 8);
        MT = o;   o += a16(size_t(NP));
        BYTES = o;
    }
};

// Multiloop-sum work of a diagonal with nls lane-sets: items qmb(ls) and
// r2(ls), each cut into np parts (split-point ranges), one or two parts per M wave
// (8-15; their global loads wait on L2, so the sums get as many waves as the
// interior loops).  Code: 0 = none, else 1 | isq << 1 | ls << 2 | pi << 4 | (np-1) << 6.
__host__ __device__ constexpr int mcode(bool isq, int ls, int pi, int np) {
    return 1 | (isq ? 2 : 0) | (ls << 2) | (pi << 4) | ((np - 1) << 6);
}
__device__ __forceinline__ int massign(int nls, int w) {
    constexpr int Q = 1, R = 0;
    if (nls >= 3) {
        // wave 11 takes two parts: qmb of lane-set 2 (the shortest) and r2 of
        // lane-set 0 (slot 3 = 11 - 8: the M loop runs massign(nls, w - 8) as a
        // wave's second part); r2 of lane-set 1 split over 12 and 13 (round 5:
        // one wave carried it whole, 123 terms where the others had <= 71)
        switch (w) {
            case 8: return mcode(Q, 0, 0, 2);
            case 9: return mcode(Q, 0, 1, 2);
            case 10: return mcode(Q, 1, 0, 1);
            case 11: return mcode(Q, 2, 0, 1);
            case 3: return mcode(R, 0, 0, 1);
            case 12: return mcode(R, 1, 0, 2);
            case 13: return mcode(R, 1, 1, 2);
            case 14: return mcode(R, 2, 0, 2);
            case 15: return mcode(R, 2, 1, 2);
            default: return 0;
        }
    }
    if (nls == 2) {
        switch (w) {
            case 8: return mcode(Q, 0, 0, 2);
            case 9: return mcode(Q, 0, 1, 2);
            case 10: return mcode(Q, 1, 0, 1);
            case 11: return mcode(R, 0, 0, 2);
            case 12: return mcode(R, 0, 1, 2);
            case 13: return mcode(R, 1, 0, 3);
            case 14: return mcode(R, 1, 1, 3);
            case 15: return mcode(R, 1, 2, 3);
            default: return 0;
        }
    }
    if (nls == 1) {
        if (w >= 8 && w < 12) return mcode(Q, 0, w - 8, 4);
        if (w >= 12 && w < 16) return mcode(R, 0, w - 12, 4);
    }
    return 0;
}

// One workgroup per (walker, outside variant).  pair_p: [W][n_pairs].
__global__ void __launch_bounds__(OX_NT, 1)
outside_ring_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, const int *mask,
                    double *pair_p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int w = blockIdx.x / ka.n_bvars, bv = blockIdx.x % ka.n_bvars;
    if (w >= W) return;
    if (mask && mask[w] != 1) return;
    const int v = ka.bvars[bv];
    const DevVariant V = ka.variants[v];
    const int N = uni(V.N);
    const OrLay Y(N);
    OxL L;
    L.yr = reinterpret_cast<float *>(smem + Y.YR);
    L.yc = nullptr;
    L.q1r = nullptr;
    L.qmc = nullptr;
    L.pl = reinterpret_cast<int *>(smem + Y.PL);
    L.qw = reinterpret_cast<float *>(smem + Y.QW);
    L.ow = reinterpret_cast<uint8_t *>(smem + Y.OW);
    L.part = reinterpret_cast<float *>(smem + Y.PART);
    L.mlp = reinterpret_cast<float *>(smem + Y.MLP);
    L.rec = reinterpret_cast<float *>(smem + Y.REC);
    L.rcnt = reinterpret_cast<int *>(smem + Y.REC + size_t(2) * OR_SETS * OX_RF * WAVE * 4);
    L.cl = reinterpret_cast<uint8_t *>(smem + Y.CL);
    uint8_t *cn = L.cl + Y.C;
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
    // OR_WPERM (diagnostic builds): physical wave -> role, to try other role / SIMD pairings
#ifdef OR_WPERM
    constexpr int wperm[OX_NW] = {OR_WPERM};
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(wperm[tid / WAVE]);
#else
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = uni(tid / WAVE);
#endif
    const int C = Y.C, NP = Y.NP;
    const DevTables &T = *ka.T;
#ifdef ADX_STAMP
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

    // ---- the proposal's inside tables (pf_ring_kernel's slot: qb, qm, qm1
    // diagonal-major, q5), at the variant's groups2 position
    const size_t B = 3 * size_t(ka.cells) + size_t(ka.Nmax) + 2;
    const size_t go = size_t(ka.bvar_slot[bv]) * B;
    const int cur = ka.cur_slot[w];
    const float *src = ka.tab + size_t(w) * 2 * ka.tab_slot + size_t(1 - cur) * ka.tab_slot + go;
    const size_t Cs = size_t(ka.cells);
    const float *qmg = src + Cs, *q1g = src + 2 * Cs;

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
              : XS->ctab[CT_FSM + 3];
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
    if (tid == 0) {
        int n = 0;
        for (int t = 0; t < ka.n_pairs && t < OX_MAXP; t++)
            if (ka.pairs[3 * t] == bv) L.pl[n++] = t | (ka.pairs[3 * t + 1] << 8) | (ka.pairs[3 * t + 2] << 16);
        L.pl[OX_MAXP] = n;
    }
    // the exterior factors G(i, j) = qb(i,j) ext(i,j), column-major, in the Y
    // region (zeroed after the exterior adjoint)
    float *G = L.yr;
    for (int k = tid; k < C + OR_SLACK; k += OX_NT) {
        if (k >= C) {
            G[k] = 0.f;
            continue;
        }
        const int jc = inv_colb(k), ic = k - colb(jc) + 1;
        const int ty = ptype(S[ic], S[jc]);
        const int cc = rtype(ty) * 25 + S[jc + 1] * 5 + S[ic - 1];
        const float e = L.dt[DT_EXT + ty * 36 + ((ic > 1) ? S[ic - 1] : 5) * 6 + ((jc < N) ? S[jc + 1] : 5)];
        G[k] = src[off(jc - ic, N) + ic - 1] * (ct[CT_INVMM + cc] * e);   // non-pairable: -0 * x = 0
    }
    __syncthreads();
    OSTAMP(0);   // loads + the exterior-factor pass

    // ---- exterior adjoint (outside_cells.hip, three lane-sets of m)
    if (wid == 0) {
        const float sig1 = XS->sig[1];
        float acc[OR_SETS] = {0.f, 0.f, 0.f};
        float val = 1.f;
        float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f;
        if (lane == 0) L.q5b[N] = 1.f;
        float g[OR_SETS] = {0.f, 0.f, 0.f};
        if (N >= 5) {
            const int cb = colb(N);
#pragma unroll
            for (int h = 0; h < OR_SETS; h++) g[h] = G[cb + min(h * WAVE + lane, N - 5)];
        }
        for (int j = N; j >= 1; j--) {
            float nx[OR_SETS] = {0.f, 0.f, 0.f};
            if (j - 1 >= 5) {
                const int cb = colb(j - 1);
#pragma unroll
                for (int h = 0; h < OR_SETS; h++) nx[h] = G[cb + min(h * WAVE + lane, j - 6)];
            }
            if (j >= 5) {
#pragma unroll
                for (int h = 0; h < OR_SETS; h++)
                    if (h * WAVE + lane <= j - 5) acc[h] = fmaf(val, g[h], acc[h]);
            }
            const int m5 = j - 5;
            float a5 = 0.f;
            if (m5 >= 0) {
                const int hs = m5 / WAVE, ls = m5 - hs * WAVE;
                const float src5 = hs == 0 ? acc[0] : hs == 1 ? acc[1] : acc[2];
                a5 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(src5), ls));
            }
            val = fmaf(sig1, val, q0);   // q5b[j-1]
            if (lane == 0) L.q5b[j - 1] = val;
            q0 = q1;
            q1 = q2;
            q2 = q3;
            q3 = a5;
#pragma unroll
            for (int h = 0; h < OR_SETS; h++) g[h] = nx[h];
        }
    }
    if (motif && wid == 1) {
        for (int o = lane + 1; o + mL - 1 <= N; o += WAVE) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) ok = S[o + k] == XS->motif_code[k];
            L.mat[o] = ok ? 1 : 0;
        }
    }
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
    for (int k = tid; k < C + OR_SLACK; k += OX_NT) L.yr[k] = 0.f;   // G's region: Y from here on
    __syncthreads();
    OSTAMP(1);   // exterior adjoint, window, rank lists

    const float mlbase_sig = XS->mlbase_sig, mlclosing = XS->mlclosing, pw1 = XS->pwml[1];
    auto cell_of = [&](int D, int ls, int &i, int &j) {
        i = 1 + ls * WAVE + lane;
        const bool valid = i <= N - D;
        if (!valid) i = N - D;
        j = i + D;
        return valid;
    };
    struct Idx {
        int cnt;
        int i[OR_SETS];
    };
    auto idx_load = [&](int D) {
        Idx X;
        X.cnt = 0;
#pragma unroll
        for (int k = 0; k < OR_SETS; k++) X.i[k] = 1;
        if (D < 4) return X;
        const int od = off(D, N);
        X.cnt = uni(cn[D]);
#pragma unroll
        for (int k = 0; k < OR_SETS; k++) {
            const int idx = k * WAVE + lane;
            const int ir = L.cl[od + min(idx, N - D - 1)];
            X.i[k] = idx < X.cnt ? ir : 1;
        }
        return X;
    };
    struct Pend {
        int cnt;
        int i[OR_SETS], ty2[OR_SETS];
        float mmin[OR_SETS], mo[OR_SETS], m23[OR_SETS];
        float4 t[OR_SETS];
    };
    auto tab_load = [&](int D, const Idx &X) {
        Pend P;
        P.cnt = X.cnt;
        const int umax = min(30, N - 3 - D);
        auto Sc = [&](int x) { return int(S[x < 0 ? 0 : (x > N + 1 ? N + 1 : x)]); };
#pragma unroll
        for (int k = 0; k < OR_SETS; k++) {
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
    auto rec_write = [&](int D, const Pend &P) {
        if (D < 4) return;
        if (lane == 0) L.rcnt[D & 1] = P.cnt;
#pragma unroll
        for (int k = 0; k < OR_SETS; k++) {
            const int idx = k * WAVE + lane;
            if (k * WAVE >= P.cnt) break;
            const bool vv = idx < P.cnt;
            float *r = L.rec + (((D & 1) * OR_SETS + k) * OX_RF) * WAVE + lane;
            r[0 * WAVE] = __int_as_float(P.i[k] | (P.ty2[k] << 8) | (vv ? (1 << 16) : 0));
            r[1 * WAVE] = P.mmin[k];
            r[2 * WAVE] = P.mo[k];
            r[3 * WAVE] = P.m23[k];
            r[4 * WAVE] = P.t[k].x;
            r[5 * WAVE] = P.t[k].y;
            r[6 * WAVE] = P.t[k].z;
            r[7 * WAVE] = P.t[k].w;
        }
    };
    constexpr int RW = 7;
    Pend pnext;
    Idx inext;
    pnext.cnt = 0;
    inext.cnt = 0;
    if (wid == RW) {
        rec_write(N - 1, tab_load(N - 1, idx_load(N - 1)));
        pnext = tab_load(N - 2, idx_load(N - 2));
        inext = idx_load(N - 3);
    }
    __syncthreads();

    auto frec_write = [&](int e, int ls) {
        if (e < 4 || ls >= (N - e + WAVE - 1) / WAVE) return;
        int i, j;
        const bool valid = cell_of(e, ls, i, j);
        const int ty = ptype(S[i], S[j]);
        const int oc = ty * 25 + S[i + 1] * 5 + S[j - 1];
        float *r = L.fr + (((e & 1) * OR_SETS + ls) * OX_FF) * WAVE + lane;
        r[0] = L.q5b[j] * L.q5[i - 1] * L.dt[DT_EXT + ty * 36 + ((i > 1) ? S[i - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
        r[WAVE] = L.dt[DT_MLS + ty * 25 + S[i - 1] * 5 + S[j + 1]];
        r[2 * WAVE] = L.dt[DT_MMI + oc];
        r[3 * WAVE] = mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
        r[4 * WAVE] = __int_as_float(ty | (oc << 8) | ((valid && ty != 0) ? (1 << 16) : 0));
    };
    // F: finalize diagonal e = d + 1, lane-set fl
    auto finalize = [&](int d, int fl) {
        const int e = d + 1;
        const int nle = (N - e + WAVE - 1) / WAVE;
        if (e > N - 1 || fl >= nle) return;
        const int pe = e & 1, pn = (e + 1) & 1;
        const int i = 1 + fl * WAVE + lane;
        if (i > N - e) return;
        const int j = i + e;
        const float *mp = L.mlp + pe * OX_NW * WAVE + lane;
        float qmbv = 0.f, r2 = 0.f;   // the parts of this lane-set's items (massign)
#pragma unroll
        for (int w2 = 0; w2 < OX_NW; w2++) {
            const int c = massign(nle, w2);
            if (c && ((c >> 2) & 3) == fl) {
                if (c & 2) qmbv += mp[w2 * WAVE];
                else r2 += mp[w2 * WAVE];
            }
        }
        const float R = i >= 2 ? pw1 * (L.rq[pn * NP + i - 1] + L.rr[pn * NP + i - 1]) : 0.f;
        const float chain = j < N ? mlbase_sig * L.r1[pn * NP + i] : 0.f;
        const float qm1b = qmbv + R + r2 + chain;
        const float *fr = L.fr + ((pe * OR_SETS + fl) * OX_FF) * WAVE + lane;
        const int tp = __float_as_int(fr[4 * WAVE]);
        float a_int = 0.f;
        const float *pp = L.part + (pe * OR_SETS + fl) * OX_NB * WAVE + lane;
#pragma unroll
        for (int b = 0; b < OR_NB; b++) a_int += pp[b * WAVE];
        if (N - 3 - e < 0) a_int = 0.f;
        L.rq[pe * NP + i] = qmbv;
        L.rr[pe * NP + i] = R;
        L.r1[pe * NP + i] = qm1b;
        L.yr[rowb(i, N) + e - 4] += qmbv;   // Y(i, j): X(i, j) was stored two diagonals ago
        float qbbm = 0.f;
        if (tp >> 16) {
            const float qbb = a_int + fr[0] + qm1b * fr[WAVE];
            qbbm = qbb * fr[2 * WAVE];
            if (e - 2 >= 4) L.yr[rowb(i + 1, N) + e - 6] = qbb * fr[3 * WAVE];   // X(i+1, j-1)
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
    // one part of a multiloop-sum item of diagonal d (massign): qmb or r2 of
    // lane-set ls, split points pi / np of the lane-set's longest range
    auto mpart = [&](int d, bool isq, int ls, int pi, int np) {
        int i = 1 + ls * WAVE + lane;
        const int ilast = min(N - d, (ls + 1) * WAVE);
        if (i > N - d) i = N - d;
        const int j = i + d;
        float acc = 0.f, acc1 = 0.f;
        constexpr int MB = 8;
        // both sums read the slot in batches of MB terms, four batches in flight
        // (a batch's global loads are issued three batches before it is summed)
        if (isq) {
            // qmb: t = 0 .. N-j-5: Y(i, j+5+t) = YR[rowb(i) + d + 1 + t] (LDS),
            // qm1(j+1, j+5+t) on diagonal t+4 at position j (slot, coalesced)
            const int lim = N - j - 5;
            const int Tq = N - (1 + ls * WAVE + d) - 4;
            const int ta = (Tq * pi) / np, tb = (Tq * (pi + 1)) / np;
            const float *py = L.yr + rowb(i, N) + d + 1;
            auto ld = [&](float (&q)[MB], int t) __attribute__((always_inline)) {
#pragma unroll
                for (int k = 0; k < MB; k++) q[k] = q1g[off(min(t + k, N - 5) + 4, N) + j];
            };
            auto use = [&](const float (&q)[MB], int t) __attribute__((always_inline)) {
                float yv[MB];
#pragma unroll
                for (int k = 0; k < MB; k++) yv[k] = py[t + k];
#pragma unroll
                for (int k = 0; k < MB; k += 2) {
                    acc = fmaf((t + k <= lim && t + k < tb) ? yv[k] : 0.f, q[k], acc);
                    acc1 = fmaf((t + k + 1 <= lim && t + k + 1 < tb) ? yv[k + 1] : 0.f, q[k + 1], acc1);
                }
            };
            float qa[MB], qb[MB], qc[MB], qd[MB];
            int t = ta;
            if (t < tb) ld(qa, t);
            if (t + MB < tb) ld(qb, t + MB);
            if (t + 2 * MB < tb) ld(qc, t + 2 * MB);
            while (t < tb) {
                if (t + 3 * MB < tb) ld(qd, t + 3 * MB);
                use(qa, t);
                t += MB;
                if (t >= tb) break;
                if (t + 3 * MB < tb) ld(qa, t + 3 * MB);
                use(qb, t);
                t += MB;
                if (t >= tb) break;
                if (t + 3 * MB < tb) ld(qb, t + 3 * MB);
                use(qc, t);
                t += MB;
                if (t >= tb) break;
                if (t + 3 * MB < tb) ld(qc, t + 3 * MB);
                use(qd, t);
                t += MB;
            }
        } else {
            // r2: u = 5 .. i-1 (ip = i - u): Y(i-u, j) = YR[rowb(i-u) + d + u - 4]
            // (LDS), qm(i-u, i-1) on diagonal u-1 at position i-u-1 (slot, coalesced)
            const int lim = i - 1;
            const int Tr = ilast - 5;
            const int ua = 5 + (Tr * pi) / np, ub = 5 + (Tr * (pi + 1)) / np;
            auto ld = [&](float (&q)[MB], int u) __attribute__((always_inline)) {
#pragma unroll
                for (int k = 0; k < MB; k++) {
                    const int uu = u + k;
                    const bool ok = uu <= lim && uu < ub;
                    q[k] = qmg[off(min(uu, N - 1) - 1, N) + (ok ? i - uu - 1 : 0)];
                }
            };
            auto use = [&](const float (&q)[MB], int u) __attribute__((always_inline)) {
                // Y(i-u-k, j): the row base moves by (i - u - k - N + 3) per term
                const int ip0 = max(i - u, 1);
                const int a0 = rowb(ip0, N) + d + u - 4;
                const int D0 = i - u - N + 3;
                float yv[MB];
#pragma unroll
                for (int k = 0; k < MB; k++) {
                    const int uu = u + k;
                    const bool ok = uu <= lim && uu < ub;
                    const int a = a0 + k * D0 - (k * (k - 1)) / 2;
                    yv[k] = L.yr[ok ? a : a0];
                    yv[k] = ok ? yv[k] : 0.f;
                }
#pragma unroll
                for (int k = 0; k < MB; k += 2) {
                    acc = fmaf(yv[k], q[k], acc);
                    acc1 = fmaf(yv[k + 1], q[k + 1], acc1);
                }
            };
            float qa[MB], qb[MB], qc[MB], qd[MB];
            int u = ua;
            if (u < ub) ld(qa, u);
            if (u + MB < ub) ld(qb, u + MB);
            if (u + 2 * MB < ub) ld(qc, u + 2 * MB);
            while (u < ub) {
                if (u + 3 * MB < ub) ld(qd, u + 3 * MB);
                use(qa, u);
                u += MB;
                if (u >= ub) break;
                if (u + 3 * MB < ub) ld(qa, u + 3 * MB);
                use(qb, u);
                u += MB;
                if (u >= ub) break;
                if (u + 3 * MB < ub) ld(qb, u + 3 * MB);
                use(qc, u);
                u += MB;
                if (u >= ub) break;
                if (u + 3 * MB < ub) ld(qc, u + 3 * MB);
                use(qd, u);
                u += MB;
            }
        }
        return acc + acc1;
    };
    auto fin = [&](int d, auto wc) {
        constexpr int w = decltype(wc)::value;
        if constexpr (w < OR_SETS) {
            finalize(d, w);
        } else if constexpr (w < 2 * OR_SETS) {
            frec_write(d, w - OR_SETS);   // diagonal d, finalized next step
        } else if (w == RW) {
            rec_write(d - 1, pnext);
            pnext = tab_load(d - 2, inext);
            inext = idx_load(d - 3);
        }
    };

    if (wid < OR_NB) {
        switch (wid) {
            // loop sizes in blocks of about equal cost (a size >= 6: 3 reads for its
            // special shapes + one per 4 generic ones per lane-set; sizes <= 5 ~3 per
            // shape), a little less on the finalize (0-2) and record (7) waves
            case 0: b_sweep<OR_SETS, 28, 20, 13, 0, -1>(L, N, lane, std::integral_constant<int, 0>{}, fin OX_STP_ARGS); break;
            case 1: b_sweep<OR_SETS, 27, 21, 1, 7, -1>(L, N, lane, std::integral_constant<int, 1>{}, fin OX_STP_ARGS); break;
            case 2: b_sweep<OR_SETS, 26, 22, 12, 6, -1>(L, N, lane, std::integral_constant<int, 2>{}, fin OX_STP_ARGS); break;
            case 3: b_sweep<OR_SETS, 4, 19, 14, -1, -1>(L, N, lane, std::integral_constant<int, 3>{}, fin OX_STP_ARGS); break;
            case 4: b_sweep<OR_SETS, 3, 24, 16, 9, -1>(L, N, lane, std::integral_constant<int, 4>{}, fin OX_STP_ARGS); break;
            case 5: b_sweep<OR_SETS, 30, 25, 18, 11, -1>(L, N, lane, std::integral_constant<int, 5>{}, fin OX_STP_ARGS); break;
            case 6: b_sweep<OR_SETS, 5, 23, 15, 8, -1>(L, N, lane, std::integral_constant<int, 6>{}, fin OX_STP_ARGS); break;
            default: b_sweep<OR_SETS, 29, 2, 17, 10, -1>(L, N, lane, std::integral_constant<int, 7>{}, fin OX_STP_ARGS); break;   // wave 7
        }
    } else for (int d = N - 1; d >= 3; d--) {
        const int nls = d >= 4 ? (N - d + WAVE - 1) / WAVE : 0;
        const int par = d & 1;
        if (d >= 4) {
            // ---------------- M: the multiloop-sum parts of diagonal d on this wave
            const int c = massign(nls, wid);
            if (c) L.mlp[(par * OX_NW + wid) * WAVE + lane] = mpart(d, (c & 2) != 0, (c >> 2) & 3, (c >> 4) & 3, (c >> 6) + 1);
            const int c2 = massign(nls, wid - OR_NB);   // a second part, in the slot of B wave wid - 8
            if (c2) L.mlp[(par * OX_NW + wid - OR_NB) * WAVE + lane] = mpart(d, (c2 & 2) != 0, (c2 >> 2) & 3, (c2 >> 4) & 3, (c2 >> 6) + 1);
        }
        OSTAMP(4);   // M sums
        lds_barrier();
        OSTAMP(6);   // barrier
    }
#ifdef ADX_STAMP
    if (lane == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_stamps_or[wid][k], st_acc[k]);
#endif
    // ---- requested pairs of this fold, the motif's inner pairs credited from
    // its closing cell (outside_cells.hip)
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

// LDS bytes of the ring outside kernel for this workload (0: not covered)
size_t outside_ring_lds(const KArgs &ka) {
    if (ka.Nmax < OR_NMIN || ka.Nmax > OR_NMAX || ka.n_pairs > OX_MAXP) return 0;
    const OrLay y(ka.Nmax);
    return y.BYTES + 256 <= 160 * 1024 ? y.BYTES : 0;
}

hipError_t launch_outside_ring(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *pair_p,
                               hipStream_t stream) {
    const size_t lds = outside_ring_lds(ka);
    if (lds == 0 || !ka.tab || !ka.bvar_slot) return hipErrorInvalidValue;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(outside_ring_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(outside_ring_kernel, dim3(W * ka.n_bvars), dim3(OX_NT), lds, stream, ka, ka.X, seqs, W, mask,
                       pair_p);
    return hipGetLastError();
}

}  // namespace adx
