// gfx950 kernels of the addapt engine: McCaskill inside partition function
// (ViennaRNA-2.x default model, dangles = 2) with dot-bracket hard constraints
// and the ligand motif, the score of MacrostateProbTerm / ScoreFunction, and
// the fused Monte Carlo step (mutation move -> PF variants -> Metropolis).
//
// Reference path (/root/reference): MonteCarlo::apply sampling.cc:55-99 ->
// ScoreFunction::evaluate scoring.cc:114-158 -> MacrostateProbTerm::evaluate
// scoring.cc:233-259 -> ViennaRnaFold::macrostate_prob scoring.cc:53-71 ->
// vrna_pf (ViennaRNA, not vendored).
//
// Execution model (DESIGN.md "Kernels"): one workgroup of NT = 512 threads
// (8 wave64) owns one walker; its DP tables qb / qm / qm1 / qbm live in LDS in
// diagonal-major order, so the cells (i, i+d) of one anti-diagonal are
// contiguous.  A diagonal is processed in two barrier-separated phases:
//   phase A  every wave takes a (cell chunk, term slice) of three jobs:
//            qb(d) interior + multiloop terms, qm(d-1) split terms, q5(d);
//            lanes = cells, so the loop over terms is wave-uniform (scalar
//            control, constant-memory term list) and the LDS reads of one
//            wave-instruction hit consecutive addresses;
//   phase B  one lane per cell sums the slices and finishes qb, qbm, qm1, qm,
//            q5, and wave 0 compacts the pairable cells of diagonal d+1.
// No MFMA: the recurrence is a sum of data-dependent products, not a dense
// contraction.  Tables are FP32 with a per-nucleotide scale sigma (ViennaRNA's
// pf_scale); ensemble energies are returned as float like vrna_pf.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.hpp"

namespace adx {

#ifdef ADX_STAMP
// Diagnostic build only: per-wave cycle sums of the per-diagonal phases
// (s_memtime), read back through adx_debug_stamps().  Never in the product.
__device__ unsigned long long g_stamps[16][16];
#define STAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

namespace {

constexpr int WAVE = 64;

// index of the first cell of diagonal dd (cells with j - i = dd >= 4)
__device__ __forceinline__ int off(int dd, int N) { return ((dd - 4) * (2 * N - 3 - dd)) >> 1; }

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Full-wave sum via DPP (quad_perm, row_shr, row_bcast): VALU-only, no LDS
// crossbar; the total lands in lane 63 and is read back with readlane.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_add(float v) {
    const int moved = __builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, false);
    return v + __int_as_float(moved);
}
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_add<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x114, 0xf>(v);  // row_shr:4
    v = dpp_add<0x118, 0xf>(v);  // row_shr:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
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
constexpr int DT_SPK = 896;    // special hairpin keys (bit patterns)
constexpr int DT_SPV = DT_SPK + MAX_SPECIAL_HP;
constexpr int DT_HP = DT_SPV + MAX_SPECIAL_HP;  // [u] hairpin length factor

// LDS carve-out for one workgroup (see lds_bytes()).
struct Lds {
    float *qbm, *qm, *qm1;
    uint8_t *cc;       // inner-pair code per cell (diagonal-major)
    float *scr;        // 2 x NT floats (double-buffered partial rows) + 4 q5 partials
    float *ct;         // CT_SIZE factor table (DevScaled::ctab)
    float *dt;         // LDS copy of per-cell tables (DT_*)
    float *q5;
    float *misc;       // [0] = q5 partial
    double *G;         // per-variant ensemble energies
    uint8_t *S, *up, *dn, *ptn, *enc, *flg, *mat;
    uint8_t *lists;    // plist[4] then pinv[4], NP bytes each
    int np;
    int *pcount;       // [2]
    uint8_t *raw;      // scored sequence (Nraw)
};

template <int NT>
__device__ Lds carve(char *base, const KArgs &ka) {
    Lds L;
    const int C = ka.cells;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        char *p = base + o;
        o += (bytes + 15) & ~size_t(15);
        return p;
    };
    L.qbm = reinterpret_cast<float *>(take(size_t(C) * 4));
    L.qm = reinterpret_cast<float *>(take(size_t(C) * 4));
    L.qm1 = reinterpret_cast<float *>(take(size_t(C) * 4));
    L.cc = reinterpret_cast<uint8_t *>(take(size_t(C)));
    L.scr = reinterpret_cast<float *>(take(2 * NT * 4 + 16));
    L.ct = reinterpret_cast<float *>(take(CT_SIZE * 4));
    L.dt = reinterpret_cast<float *>(take(size_t(DT_HP + ka.Nmax + 1) * 4));
    const int NP = ka.Nmax + 2;
    L.q5 = reinterpret_cast<float *>(take(NP * 4));
    L.misc = reinterpret_cast<float *>(take(16 * 4));
    L.G = reinterpret_cast<double *>(take(ka.n_variants * 8));
    L.pcount = reinterpret_cast<int *>(take(4 * 4));
    L.S = reinterpret_cast<uint8_t *>(take(NP));
    L.up = reinterpret_cast<uint8_t *>(take(NP));
    L.dn = reinterpret_cast<uint8_t *>(take(NP));
    L.ptn = reinterpret_cast<uint8_t *>(take(NP));
    L.enc = reinterpret_cast<uint8_t *>(take(NP));
    L.flg = reinterpret_cast<uint8_t *>(take(NP));
    L.mat = reinterpret_cast<uint8_t *>(take(NP));
    L.np = NP;
    L.lists = reinterpret_cast<uint8_t *>(take(8 * NP));
    L.raw = reinterpret_cast<uint8_t *>(take(NP));
    return L;
}

template <int NT>
__device__ void load_ctab(const KArgs &ka, const Lds &L) {
    for (int k = threadIdx.x; k < CT_SIZE; k += NT) L.ct[k] = ka.X->ctab[k];
    const DevTables &T = *ka.T;
    const DevScaled &X = *ka.X;
    for (int k = threadIdx.x; k < 200; k += NT) {
        L.dt[DT_MMH + k] = (&T.mmH[0][0][0])[k];
        L.dt[DT_MMI + k] = (&T.mmI[0][0][0])[k];
        L.dt[DT_MLS + k] = (&T.mlstem[0][0][0])[k];
    }
    for (int k = threadIdx.x; k < 288; k += NT) L.dt[DT_EXT + k] = (&T.ext[0][0][0])[k];
    for (int k = threadIdx.x; k < 8; k += NT) L.dt[DT_TAU + k] = T.termAU[k];
    for (int k = threadIdx.x; k < MAX_SPECIAL_HP; k += NT) {
        L.dt[DT_SPK + k] = __uint_as_float(k < X.n_special ? X.sp_key[k] : 0u);
        L.dt[DT_SPV + k] = X.sp_val[k];
    }
    for (int k = threadIdx.x; k <= ka.Nmax; k += NT) L.dt[DT_HP + k] = X.hp[k];
}

__device__ __forceinline__ uint8_t *plist(const Lds &L, int b) { return L.lists + b * L.np; }
__device__ __forceinline__ uint8_t *pinv(const Lds &L, int b) { return L.lists + (4 + b) * L.np; }

// ---------------------------------------------------------------- hard constraints
// flg bits: 1 = 'x' (no pair), 2 = '<' (pairs upstream), 4 = '>' (downstream);
// ptn = enforced partner (0 none); enc = innermost enclosing enforced pair id.
__device__ __forceinline__ bool allowed(const Lds &L, int i, int j) {
    const int fi = L.flg[i], fj = L.flg[j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[i], pj = L.ptn[j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[i] == L.enc[j];
}

__device__ __forceinline__ bool pairable(const Lds &L, int i, int j) {
    return ptype(L.S[i], L.S[j]) != 0 && allowed(L, i, j);
}

// one wave: compact the pairable cells of diagonal dd into buffer b
__device__ void build_plist(const Lds &L, int N, int dd, int b, int lane) {
    const int c = N - dd;
    int base = 0;
    for (int r0 = 0; r0 < c; r0 += WAVE) {
        const int r = r0 + lane;
        const int i = r + 1;
        const bool valid = r < c;
        const bool f = valid && pairable(L, i, i + dd);
        const unsigned long long m = __ballot(f);
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        if (f) {
            plist(L, b)[base + rank] = static_cast<uint8_t>(i);
            pinv(L, b)[i] = static_cast<uint8_t>(base + rank);
        } else if (valid) {
            pinv(L, b)[i] = 0xFF;
        }
        base += __popcll(m);
    }
    if (lane == 0) L.pcount[b] = base;
}

// ---------------------------------------------------------------- inside PF
// Per-diagonal pipeline with ONE barrier per iteration d:
//   jobs (all waves, lanes = cells):  A  qb(d) partials      (reads spans <= d-2)
//                                     B  qm(d-2) partials    (qm1 span d-2, qm <= d-7)
//                                     C  q5[d-1] partial     (qb spans <= d-2)
//   finalize (one item per thread):   qb(d-1) + qbm/code + qm1(d-1), qm(d-3), q5[d-2],
//                                     from the partials iteration d-1 left in the other
//                                     scratch buffer; plus the pairable list of d+1.
// qb(d) never reads span d-1 (stack = span d-2), so the finalize of d-1 and the
// partials of d share one phase.
template <int NT>
__device__ double pf_inside(const KArgs &ka, int v, const uint8_t *raw, const Lds &L,
                           const DevScaled *__restrict__ XS) {
    constexpr int NW = NT / WAVE;
    const DevVariant V = ka.variants[v];
    const int N = V.N;
    const DevTables &T = *ka.T;
    const DevScaled &X = *ka.X;
    const float *ct = L.ct;
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);

    // ---- per-variant setup: sequence, constraint arrays, motif sites
    const uint8_t *cons = ka.cons + V.cons_off;
    const int np = N + 2;
    const uint8_t *bef = nullptr, *aft = nullptr;
    int blen = 0;
    if (V.ctx >= 0) {
        bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
        blen = ka.ctx_off[4 * V.ctx + 1];
        aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
    }
    bool constrained = false;
    for (int k = tid; k < np; k += NT) {
        uint8_t s = 0;
        if (k >= 1 && k <= N) {
            const int p = k - 1;
            if (p < blen) s = bef[p];
            else if (p < blen + ka.Nraw) s = raw[p - blen];
            else s = aft[p - blen - ka.Nraw];
        }
        L.S[k] = s;
        const uint8_t f = cons[4 * np + k], pt = cons[2 * np + k];
        L.up[k] = cons[k];
        L.dn[k] = cons[np + k];
        L.ptn[k] = pt;
        L.enc[k] = cons[3 * np + k];
        L.flg[k] = f;
        L.mat[k] = 0;
        if (k >= 1 && k <= N && (f || pt)) constrained = true;
    }
    constrained = __syncthreads_or(constrained);
    if (tid == 0) {
        // ViennaRNA's S1 wrap-around (only reaches values that are never used)
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
        L.q5[0] = 1.0f;
    }
    const int mL = X.motif_len;
    if (V.motif && mL > 0) {
        for (int o = tid + 1; o + mL - 1 <= N; o += NT) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) {
                if (L.S[o + k] != X.motif_code[k]) ok = false;
            }
            for (int k = 0; k < mL && ok; k++) {
                const int pk = X.motif_pt[k];
                if (pk < 0) ok = L.up[o + k] >= 1;
                else if (pk > k) ok = allowed(L, o + k, o + pk);
            }
            L.mat[o] = ok ? 1 : 0;
        }
    }
    __syncthreads();
    const float sig1 = X.sig[1];
    if (tid == 0) {
        for (int j = 1; j <= 3 && j <= N; j++) L.q5[j] = (L.up[j] >= 1) ? L.q5[j - 1] * sig1 : 0.f;
    }
    if (wid == NW - 1 && N - 1 >= 4) build_plist(L, N, 4, 0, lane);
    __syncthreads();

    const float mlbase_sig = X.mlbase_sig;
    const float mlclosing = X.mlclosing;
    const float eTAU = ct[CT_FSM + 6];
    const int mlen = V.motif ? mL : 0;
    const float mextra = X.motif_extra;
    const int nsp = X.n_special < MAX_SPECIAL_HP ? X.n_special : MAX_SPECIAL_HP;
    // split of the previous iteration (to find its partials)
    int p_gA = 0, p_slA = 0, p_gB = 0, p_slB = 0, p_nA = 0;
#ifdef ADX_STAMP
    unsigned long long st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

    for (int d = 4; d <= N + 2; ++d) {
        STAMP(10);
        const int buf = d & 1;
        float *scr = L.scr + buf * NT;
        const float *pscr = L.scr + (buf ^ 1) * NT;
        float *scrC = L.scr + 2 * NT;
        // ---------------- finalize items of the previous iteration
        const int df = d - 1;                     // qb diagonal to finish
        const int cdf = (df >= 4 && df <= N - 1) ? N - df : 0;
        const int dq = d - 3;                     // qm diagonal to finish
        const int cq = (dq >= 4 && dq <= N - 6) ? N - dq : 0;
        const int jq = d - 2;                     // q5 index to finish
        if (tid < cdf) {
            const int i = tid + 1, j = i + df;
            const int idx = off(df, N) + i - 1;
            const int r = pinv(L, df & 3)[i];
            const int si = L.S[i], sj = L.S[j];
            const int sim = L.S[i - 1], sjp = L.S[j + 1];
            const int btype = ptype(si, sj);
            float qbv = 0.f;
            if (r != 0xFF) {
                const int ch = r / WAVE, ln = r % WAVE;
                for (int sl = 0; sl < p_slA; sl++) qbv += pscr[(sl * p_gA + ch) * WAVE + ln];
                const int u = df - 1;
                if (L.up[i + 1] >= u) {
                    float h = -1.f;
                    if (u == 3 || u == 4 || u == 6) {
                        const uint32_t key = hp_key(L.S, i, u + 2);
                        for (int k = 0; k < nsp; k++)
                            if (__float_as_uint(L.dt[DT_SPK + k]) == key) { h = L.dt[DT_SPV + k]; break; }
                    }
                    if (h < 0.f)
                        h = L.dt[DT_HP + u] * ((u == 3) ? L.dt[DT_TAU + btype]
                                                        : L.dt[DT_MMH + btype * 25 + L.S[i + 1] * 5 + L.S[j - 1]]);
                    qbv += h;
                }
                if (df == mlen - 1 && L.mat[i]) qbv += mextra;
            }
            const int code = rtype(btype) * 25 + sjp * 5 + sim;
            L.qbm[idx] = qbv * L.dt[DT_MMI + code];
            L.cc[idx] = static_cast<uint8_t>(code);
            if (df <= N - 6) {
                float q1 = qbv * L.dt[DT_MLS + btype * 25 + sim * 5 + sjp];
                if (df >= 5 && L.up[j] >= 1) q1 = fmaf(L.qm1[colb(j - 1) + i - 1], mlbase_sig, q1);
                L.qm1[colb(j) + i - 1] = q1;
            }
        } else if (tid < cdf + cq) {
            const int r = tid - cdf;
            const int ch = r / WAVE, ln = r % WAVE;
            float sq = 0.f;
            for (int sl = 0; sl < p_slB; sl++) sq += pscr[(p_nA + sl * p_gB + ch) * WAVE + ln];
            L.qm[rowb(r + 1, N) + dq - 4] = sq;
        } else if (tid == cdf + cq && jq >= 4 && jq <= N) {
            L.q5[jq] = ((L.up[jq] >= 1) ? L.q5[jq - 1] * sig1 : 0.f) + scrC[jq & 1];
        }
        if (wid == NW - 1 && d + 1 <= N - 1) build_plist(L, N, d + 1, (d + 1) & 3, lane);
        STAMP(0);

        // ---------------- jobs
        const bool jobA = d <= N - 1;
        const int dbq = d - 2;
        const bool jobB = dbq >= 4 && dbq <= N - 6;
        const int cp = jobA ? L.pcount[d & 3] : 0;
        const int cb = jobB ? N - dbq : 0;
        const int gA = (cp + WAVE - 1) / WAVE;
        const int gB = (cb + WAVE - 1) / WAVE;
        const int umax = d - 6 < 30 ? d - 6 : 30;
        // job A term list per cell: [7 small shapes | generic (u = 6..umax, n1 = 2..u-2)
        // | multiloop closing (tp = 6..d-5) | umax bulge pairs | umax-3 1xn pairs]
        const int nGen = umax >= 6 ? ((umax - 3) * (umax - 2)) / 2 - 3 : 0;
        const int nML = d > 10 ? d - 10 : 0;
        const int nBul = umax > 0 ? umax : 0;
        const int n1n = umax > 3 ? umax - 3 : 0;
        const int nT = 7 + nGen + nML + nBul + n1n;
        const int nB = jobB ? dbq - 3 : 0;
        int nA = 0;
        if (gA && gB) {
            const int wA = gA * (6 + nGen + nML + 3 * (nBul + n1n));
            const int wB = gB * 2 * nB;
            nA = (NW * wA + (wA + wB) / 2) / (wA + wB);
            if (nA < gA) nA = gA;
            if (nA > NW - gB) nA = NW - gB;
        } else if (gA) {
            nA = NW;
        }
        const int slA = gA ? nA / gA : 0;
        const int slB = gB ? (NW - nA) / gB : 0;

        if (wid < gA * slA) {
            // ====================== job A: qb(d) partials
            const int ch = wid % gA, sl = wid / gA;
            const int r = ch * WAVE + lane;
            const bool active = r < cp;
            const int i = plist(L, d & 3)[active ? r : 0];
            const int j = i + d;
            const int type = ptype(L.S[i], L.S[j]);
            const int si1 = L.S[i + 1], sj1 = L.S[j - 1];
            const int A_ = L.up[i + 1], B_ = L.dn[j - 1];
            const int ocode = type * 25 + si1 * 5 + sj1;
            const float mmI_ij = L.dt[DT_MMI + ocode];
            const float mlc_ij = L.dt[DT_MLS + rtype(type) * 25 + sj1 * 5 + si1];
            const bool free_cell = !active || (A_ >= umax && B_ >= umax);
            const bool masked = constrained && (__ballot(!free_cell) != 0ull);
            const int t0 = (sl * nT) / slA, t1 = ((sl + 1) * nT) / slA;
            const float tau_ij = type > 2 ? eTAU : 1.f;
            // ---- small shapes: int11/21/22 come from HBM/L2, so they are issued
            // first and consumed after the LDS-bound loops
            float smq[7], smf[7];
#pragma unroll
            for (int s = 0; s < 7; s++) {
                smq[s] = 0.f;
                smf[s] = 0.f;
                const int n1 = (s == 0) ? 0 : (s == 1 || s == 2) ? 1 : (s == 6) ? 3 : 2;
                const int n2 = (s == 0) ? 0 : (s == 1 || s == 3) ? 1 : (s == 2 || s == 4 || s == 6) ? 2 : 3;
                const int u = n1 + n2;
                if (s >= t0 && s < t1 && u <= umax) {
                    const int ix = off(d - 2 - u, N) + i + n1;
                    const int code = L.cc[ix];
                    const int t2 = (code * 41) >> 10;
                    const int p = i + 1 + n1, q = j - 1 - n2;
                    const int sp1 = L.S[p - 1], sq1 = L.S[q + 1];
                    const bool ok = !masked || ((n1 <= A_) & (n2 <= B_));
                    smq[s] = ok ? L.qbm[ix] * ct[CT_INVMM + code] : 0.f;
                    if (s == 0) smf[s] = ct[CT_STK + type * 8 + t2] * ct[CT_FSM + 0];
                    else if (s == 1) smf[s] = T.int11[type][t2][si1][sj1] * ct[CT_FSM + 2];
                    else if (s == 2) smf[s] = T.int21[type][t2][si1][sq1][sj1] * ct[CT_FSM + 3];
                    else if (s == 3) smf[s] = T.int21[t2][type][sq1][si1][sp1] * ct[CT_FSM + 3];
                    else if (s == 4) smf[s] = T.int22[type][t2][si1][sp1][sq1][sj1] * ct[CT_FSM + 4];
                    else smf[s] = ct[CT_M23O + ocode] * ct[CT_M23O + code] * ct[CT_FSM + 5];
                }
            }
            STAMP(1);
            float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#ifndef ADX_ABL_GENERIC
            // ---- generic interior loops: contiguous n1 runs of one u per row
            {
                const int gs = (t0 > 7 ? t0 : 7) - 7, ge = (t1 < 7 + nGen ? t1 : 7 + nGen) - 7;
                if (gs < ge) {
                    int u = 6, rs = 0;
                    while (rs + (u - 3) <= gs) { rs += u - 3; u++; }
                    int idx = gs;
                    while (idx < ge) {
                        const int a = 2 + (idx - rs);
                        const int rowend = rs + (u - 3);
                        const int e = (ge < rowend ? ge : rowend) - rs + 2;  // n1 in [a, e)
                        const float *fr = XS->fgen + (u - 6) * FG_ROW - 2;    // fr[n1] (scalar loads)
                        const float *q = L.qbm + off(d - 2 - u, N) + i;  // q[n1] = qbm(i+1+n1, j-1-u+n1)
                        int n1 = a;
                        if (!masked) {
                            for (; n1 + 8 <= e; n1 += 8) {
                                float qv[8], fv[8];
#pragma unroll
                                for (int k = 0; k < 8; k++) { qv[k] = q[n1 + k]; fv[k] = fr[n1 + k]; }
#pragma unroll
                                for (int k = 0; k < 8; k++) g[k] = fmaf(qv[k], fv[k], g[k]);
                            }
                            for (; n1 + 2 <= e; n1 += 2) {
                                const float q0 = q[n1], q1 = q[n1 + 1];
                                g[0] = fmaf(q0, fr[n1], g[0]);
                                g[1] = fmaf(q1, fr[n1 + 1], g[1]);
                            }
                            if (n1 < e) g[2] = fmaf(q[n1], fr[n1], g[2]);
                        } else {
                            const int lo = u - B_;  // n2 <= B_  <=>  n1 >= u - B_
                            for (; n1 + 4 <= e; n1 += 4) {
                                float qv[4];
#pragma unroll
                                for (int k = 0; k < 4; k++) qv[k] = q[n1 + k];
#pragma unroll
                                for (int k = 0; k < 4; k++) {
                                    const bool ok = (n1 + k <= A_) & (n1 + k >= lo);
                                    g[k] = fmaf(qv[k], ok ? fr[n1 + k] : 0.f, g[k]);
                                }
                            }
                            for (; n1 < e; n1++) {
                                const bool ok = (n1 <= A_) & (n1 >= lo);
                                g[4] = fmaf(q[n1], ok ? fr[n1] : 0.f, g[4]);
                            }
                        }
                        idx = rs + (e - 2);
                        rs = rowend;
                        u++;
                    }
                }
            }
#endif
            STAMP(2);
            float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#ifndef ADX_ABL_ML
            // ---- multiloop closed by (i,j): qm[i+1][k-1] * qm1[k][j-1], k = i + tp
            {
                const int b0 = 7 + nGen;
                const int ms = (t0 > b0 ? t0 : b0) - b0, me = (t1 < b0 + nML ? t1 : b0 + nML) - b0;
                if (ms < me) {
                    const float *qa = L.qm + rowb(i + 1, N);          // qa[m] = qm[i+1][i+tp-1], tp = 6 + m
                    const float *qb1 = L.qm1 + colb(j - 1) + i + 5;   // qb1[m] = qm1[i+tp][j-1]
                    int mm = ms;
                    for (; mm + 8 <= me; mm += 8) {
                        float av[8], bv[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) { av[k] = qa[mm + k]; bv[k] = qb1[mm + k]; }
#pragma unroll
                        for (int k = 0; k < 8; k++) m[k] = fmaf(av[k], bv[k], m[k]);
                    }
                    for (; mm < me; mm++) m[0] = fmaf(qa[mm], qb1[mm], m[0]);
                }
            }
#endif
            STAMP(3);
            float sA = 0.f, sB = 0.f, sC = 0.f, sD = 0.f;
#ifndef ADX_ABL_SPECIAL
            {
                const int b0 = 7 + nGen + nML;
                // bulges (0,n) and (n,0), n = 1..umax: unit n - 1 covers both sides
                {
                    const int bs = (t0 > b0 ? t0 : b0) - b0;
                    const int be = (t1 < b0 + nBul ? t1 : b0 + nBul) - b0;
                    int n = bs + 1;
                    int o = off(d - 2 - n, N) + i;  // cell (i+1, j-1-n)
                    if (n == 1 && n <= be) {
                        const int c0 = L.cc[o], c1 = L.cc[o + 1];
                        const float v0 = L.qbm[o], v1 = L.qbm[o + 1];
                        const float f0 = ct[CT_FSM + 1];
                        const float x0 = ct[CT_INVMM + c0] * ct[CT_STK + type * 8 + ((c0 * 41) >> 10)] * f0;
                        const float x1 = ct[CT_INVMM + c1] * ct[CT_STK + type * 8 + ((c1 * 41) >> 10)] * f0;
                        const bool ok0 = !masked || (1 <= B_), ok1 = !masked || (1 <= A_);
                        sA = fmaf(v0, ok0 ? x0 : 0.f, sA);
                        sB = fmaf(v1, ok1 ? x1 : 0.f, sB);
                        o -= N - (d - 4);  // off(D-1) = off(D) - (N - D + 1), D = d-3
                        n++;
                    }
                    // two units per iteration: 4 independent cc/qbm loads in flight
                    for (; n + 1 <= be; n += 2) {
                        const int o2 = o - (N - (d - 3 - n));
                        const int c0 = L.cc[o], c1 = L.cc[o + n], c2 = L.cc[o2], c3 = L.cc[o2 + n + 1];
                        const float v0 = L.qbm[o], v1 = L.qbm[o + n], v2 = L.qbm[o2], v3 = L.qbm[o2 + n + 1];
                        const float fb0 = XS->ctab[CT_FB + n] * tau_ij, fb1 = XS->ctab[CT_FB + n + 1] * tau_ij;
                        const float x0 = ct[CT_BUL + c0] * fb0, x1 = ct[CT_BUL + c1] * fb0;
                        const float x2 = ct[CT_BUL + c2] * fb1, x3 = ct[CT_BUL + c3] * fb1;
                        const bool ok0 = !masked || (n <= B_), ok1 = !masked || (n <= A_);
                        const bool ok2 = !masked || (n + 1 <= B_), ok3 = !masked || (n + 1 <= A_);
                        sA = fmaf(v0, ok0 ? x0 : 0.f, sA);
                        sB = fmaf(v1, ok1 ? x1 : 0.f, sB);
                        sC = fmaf(v2, ok2 ? x2 : 0.f, sC);
                        sD = fmaf(v3, ok3 ? x3 : 0.f, sD);
                        o = o2 - (N - (d - 4 - n));
                    }
                    if (n <= be) {
                        const int c0 = L.cc[o], c1 = L.cc[o + n];
                        const float fb = ct[CT_FB + n] * tau_ij;
                        const bool ok0 = !masked || (n <= B_), ok1 = !masked || (n <= A_);
                        sA = fmaf(L.qbm[o], ok0 ? ct[CT_BUL + c0] * fb : 0.f, sA);
                        sB = fmaf(L.qbm[o + n], ok1 ? ct[CT_BUL + c1] * fb : 0.f, sB);
                    }
                }
                // 1 x nl and nl x 1, nl = 3..umax-1: unit nl - 3 covers both sides
                {
                    const int s0 = b0 + nBul;
                    const int bs = (t0 > s0 ? t0 : s0) - s0, be = t1 - s0;
                    if (bs < be) {
                        const float mo = ct[CT_ONEN + ocode] * mmI_ij;  // outer mismatch_1n
                        int nl = bs + 3;
                        const int nle = be + 3;
                        int o = off(d - 3 - nl, N) + i;  // cell (i+2, j-1-nl) at o + 1
                        for (; nl + 1 < nle; nl += 2) {
                            const int o2 = o - (N - (d - 4 - nl));
                            const int c0 = L.cc[o + 1], c1 = L.cc[o + nl], c2 = L.cc[o2 + 1], c3 = L.cc[o2 + nl + 1];
                            const float v0 = L.qbm[o + 1], v1 = L.qbm[o + nl];
                            const float v2 = L.qbm[o2 + 1], v3 = L.qbm[o2 + nl + 1];
                            const float f0 = XS->ctab[CT_F1N + nl] * mo, f1 = XS->ctab[CT_F1N + nl + 1] * mo;
                            const bool ok0 = !masked || ((1 <= A_) & (nl <= B_));
                            const bool ok1 = !masked || ((nl <= A_) & (1 <= B_));
                            const bool ok2 = !masked || ((1 <= A_) & (nl + 1 <= B_));
                            const bool ok3 = !masked || ((nl + 1 <= A_) & (1 <= B_));
                            sA = fmaf(v0, ok0 ? ct[CT_ONEN + c0] * f0 : 0.f, sA);
                            sB = fmaf(v1, ok1 ? ct[CT_ONEN + c1] * f0 : 0.f, sB);
                            sC = fmaf(v2, ok2 ? ct[CT_ONEN + c2] * f1 : 0.f, sC);
                            sD = fmaf(v3, ok3 ? ct[CT_ONEN + c3] * f1 : 0.f, sD);
                            o = o2 - (N - (d - 5 - nl));
                        }
                        if (nl < nle) {
                            const int c0 = L.cc[o + 1], c1 = L.cc[o + nl];
                            const float f0 = ct[CT_F1N + nl] * mo;
                            const bool ok0 = !masked || ((1 <= A_) & (nl <= B_));
                            const bool ok1 = !masked || ((nl <= A_) & (1 <= B_));
                            sA = fmaf(L.qbm[o + 1], ok0 ? ct[CT_ONEN + c0] * f0 : 0.f, sA);
                            sB = fmaf(L.qbm[o + nl], ok1 ? ct[CT_ONEN + c1] * f0 : 0.f, sB);
                        }
                    }
                }
            }
#endif
            float sm = 0.f;
#pragma unroll
            for (int s = 0; s < 7; s++) sm = fmaf(smq[s], smf[s], sm);
            const float gsum = ((g[0] + g[1]) + (g[2] + g[3])) + ((g[4] + g[5]) + (g[6] + g[7]));
            const float msum = ((m[0] + m[1]) + (m[2] + m[3])) + ((m[4] + m[5]) + (m[6] + m[7]));
            const float part = ((sA + sB) + (sC + sD)) + sm + gsum * mmI_ij + msum * (mlclosing * mlc_ij);
            scr[wid * WAVE + lane] = part;
            STAMP(4);
        } else if (wid >= nA && wid < nA + gB * slB) {
            // ====================== job B: qm(dbq) partials
            // qm[i][jb] = sum_t (pre(t) + qm[i][i+t-1]) * qm1[i+t][jb]
            const int lw = wid - nA;
            const int ch = lw % gB, sl = lw / gB;
            const int r = ch * WAVE + lane;
            const bool active = r < cb;
            const int i = (active ? r : 0) + 1;
            const int jb = i + dbq;
            const int upi = L.up[i];
            const int t0 = (sl * nB) / slB, t1 = ((sl + 1) * nB) / slB;
            const float *q1 = L.qm1 + colb(jb) + i - 1;   // q1[t] = qm1[i+t][jb]
            const float *qr = L.qm + rowb(i, N) - 5;      // qr[t] = qm[i][i+t-1], t >= 5
            float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            int t = t0;
            for (; t < t1 && t < 5; t++) a[0] = fmaf((t <= upi) ? XS->pwml[t] : 0.f, q1[t], a[0]);
            if (!constrained) {
                for (; t + 8 <= t1; t += 8) {
                    float pv[8], rv[8], qv[8];
#pragma unroll
                    for (int k = 0; k < 8; k++) { pv[k] = XS->pwml[t + k]; rv[k] = qr[t + k]; qv[k] = q1[t + k]; }
#pragma unroll
                    for (int k = 0; k < 8; k++) a[k] = fmaf(pv[k] + rv[k], qv[k], a[k]);
                }
            }
            for (; t < t1; t++) a[1] = fmaf(((t <= upi) ? XS->pwml[t] : 0.f) + qr[t], q1[t], a[1]);
            scr[wid * WAVE + lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
            STAMP(5);
        }
        if (wid == NW - 1 && d - 1 >= 4 && d - 1 <= N) {
            // ====================== job C: q5[j] partial, j = d-1
            const int j = d - 1;
            float extf[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int k = 1 + lane + c * WAVE;
                extf[c] = 0.f;
                if (k <= j - 4) {
                    const int type = ptype(L.S[k], L.S[j]);
                    extf[c] = L.dt[DT_EXT + type * 36 + ((k > 1) ? L.S[k - 1] : 5) * 6 + ((j < N) ? L.S[j + 1] : 5)];
                }
            }
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const int k = 1 + lane + c * WAVE;
                if (k <= j - 4) {
                    const int ix = off(j - k, N) + k - 1;
                    acc = fmaf(L.q5[k - 1] * L.qbm[ix], ct[CT_INVMM + L.cc[ix]] * extf[c], acc);
                }
            }
            acc = wave_sum(acc);
            if (lane == 0) scrC[j & 1] = acc;
            STAMP(6);
        }
        p_gA = gA;
        p_slA = slA;
        p_gB = gB;
        p_slB = slB;
        p_nA = nA;
        STAMP(8);
        __syncthreads();
        STAMP(9);
    }
#ifdef ADX_STAMP
    if (lane == 0 && wid < 16)
        for (int k = 0; k < 12; k++) atomicAdd(&g_stamps[wid][k], st_acc[k]);
#endif
    const float z = L.q5[N];
    const double lnZ = log(static_cast<double>(z)) - N * X.log_sigma;
    return -X.kT * lnZ;
}

// ---------------------------------------------------------------- scoring
// lane 0 of the block: score from the per-variant energies in L.G
__device__ double combine_score(const KArgs &ka, const Lds &L, double *terms_out) {
    const DevScaled &X = *ka.X;
    double score = 0.0;
    for (int c = 0; c < ka.n_ctx_eff; c++) {
        for (int t = 0; t < ka.n_terms; t++) {
            const DevTermMap m = ka.tmap[c * ka.n_terms + t];
            // vrna_pf returns float (scoring.cc:58,65)
            const double gt = static_cast<double>(static_cast<float>(L.G[m.vfree]));
            const double ga = static_cast<double>(static_cast<float>(L.G[m.vcons]));
            double p = exp((gt - ga) / X.kT);
            if (!m.favorable) p = 1.0 - p;
            const double val = log(p);
            if (terms_out) terms_out[c * ka.n_terms + t] = val;
            score += m.weight * val;
        }
    }
    return score;
}

template <int NT>
__device__ double score_sequence(const KArgs &ka, const DevScaled *__restrict__ XS,
                                 const uint8_t *raw, const Lds &L,
                                 float *dG_out, double *terms_out) {
    for (int v = 0; v < ka.n_variants; v++) {
        const double g = pf_inside<NT>(ka, v, raw, L, XS);
        if (threadIdx.x == 0) {
            L.G[v] = g;
            if (dG_out) dG_out[v] = static_cast<float>(g);
        }
    }
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) s = combine_score(ka, L, terms_out);
    return s;
}

template <int NT>
__global__ void __launch_bounds__(NT, 4)
score_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, double *scores,
             double *terms, float *dG, const int *mask) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Lds L = carve<NT>(smem, ka);
    const int w = blockIdx.x;
    if (w >= W) return;
    if (mask && mask[w] != 1) return;  // MC: only walkers whose proposal changed
    load_ctab<NT>(ka, L);
    for (int k = threadIdx.x; k < ka.Nraw; k += NT) L.raw[k] = seqs[size_t(w) * ka.Nraw + k];
    __syncthreads();
    const int nt = ka.n_terms * ka.n_ctx_eff;
    const double s = score_sequence<NT>(ka, XS, L.raw, L, dG ? dG + size_t(w) * ka.n_variants : nullptr,
                                             terms ? terms + size_t(w) * nt : nullptr);
    if (threadIdx.x == 0) scores[w] = s;
}

// ---------------------------------------------------------------- mt19937
__device__ void mt_twist_wave(uint32_t *mt, int lane) {
    // three dependency-free phases (see DESIGN.md "RNG")
    for (int i = lane; i < 227; i += WAVE) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
        const uint32_t v = mt[i + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        mt[i] = v;
    }
    for (int i = 227 + lane; i < 454; i += WAVE) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
        const uint32_t v = mt[i - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        mt[i] = v;
    }
    for (int i = 454 + lane; i < 624; i += WAVE) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
        const uint32_t v = mt[i - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        mt[i] = v;
    }
}

struct MtView {
    uint32_t *mt;
    int idx;
    bool twisted;
};

__device__ uint32_t mt_next(MtView &g, int lane) {
    if (g.idx >= 624) {
        mt_twist_wave(g.mt, lane);
        g.idx = 0;
        g.twisted = true;
    }
    uint32_t y = g.mt[g.idx];
    g.idx++;
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// libstdc++-11 uniform_int_distribution (Lemire) for [0, R-1]
__device__ uint32_t mt_uniform(MtView &g, uint32_t R, int lane) {
    uint64_t product = uint64_t(mt_next(g, lane)) * R;
    uint32_t low = uint32_t(product);
    if (low < R) {
        const uint32_t threshold = (0u - R) % R;
        while (low < threshold) {
            product = uint64_t(mt_next(g, lane)) * R;
            low = uint32_t(product);
        }
    }
    return uint32_t(product >> 32);
}

__device__ double mt_canonical(MtView &g, int lane) {
    const double r = 4294967296.0;
    double sum = double(mt_next(g, lane));
    sum += double(mt_next(g, lane)) * r;
    double ret = sum / (r * r);
    if (ret >= 1.0) ret = 0.99999999999999989;  // nextafter(1, 0)
    return ret;
}

// ---------------------------------------------------------------- MC step
// One MonteCarlo::apply iteration (sampling.cc:55-99) = three launches on one
// stream: propose_kernel (thermostat, RNG streams, mutation move, unchanged
// check; one wave per walker) -> score_kernel masked to the walkers whose
// sequence changed -> accept_kernel (Metropolis, one thread per walker).
// Splitting keeps the fold kernel's register allocation free of the MC state.
__global__ void __launch_bounds__(64) propose_kernel(StepArgs st, long long step, int s) {
    const int w = blockIdx.x;
    const int lane = threadIdx.x;
    if (w >= st.W) return;
    if (st.err[w]) {
        if (lane == 0) st.changed[w] = 0;
        return;
    }
    __shared__ uint32_t mt[2 * MT_WORDS];
    uint8_t *cur = st.cur_seq + size_t(w) * st.Nraw;
    uint32_t *gA = st.mtA + size_t(w) * MT_WORDS;
    uint32_t *gC = st.mtC + size_t(w) * MT_WORDS;
    // ---- thermostat (sampling.cc:59; 309-401)
    double T;
    if (st.thermo_kind == 0) {
        T = st.t_fixed;
    } else if (st.thermo_kind == 1) {
        const int Nc = st.cycle_len;
        T = ((st.t_lo - st.t_hi) / Nc) * double(int(step % Nc)) + st.t_hi;
    } else {
        double *tr = st.train + size_t(w) * st.period;
        const int n = st.ntrain[w] + 1;
        if (lane == 0) tr[n - 1] = st.last_diff[w];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        T = st.auto_T[w];
        if (n >= st.period) {
            // nth_element(n/2): a value whose rank window covers n/2
            const int k = n / 2;
            double found = 0.0;
            bool have = false;
            for (int e = lane; e < n; e += WAVE) {
                const double x = tr[e];
                int less = 0, eq = 0;
                for (int f = 0; f < n; f++) {
                    const double y = tr[f];
                    less += (y < x);
                    eq += (y == x);
                }
                if (less <= k && k < less + eq) { found = x; have = true; }
            }
            const unsigned long long m = __ballot(have);
            const int src = m ? __ffsll((long long)m) - 1 : 0;
            const double med = __shfl(found, src, WAVE);
            const double t = med / log(st.target_rate);
            T = t > 0.0 ? t : 0.0;
            if (lane == 0) {
                st.auto_T[w] = T;
                st.ntrain[w] = 0;
            }
        } else if (lane == 0) {
            st.ntrain[w] = n;
        }
    }
    // ---- move: stream A (and C if the step will be scored)
    uint32_t *mA = mt, *mC = mt + MT_WORDS;
    for (int k = lane; k < 624; k += WAVE) {
        mA[k] = gA[k];
        mC[k] = gC[k];
    }
    __syncthreads();
    MtView a{mA, int(gA[624]), false}, c{mC, int(gC[624]), false};
    const int pick = int(mt_uniform(a, uint32_t(st.M), lane));
    const int bcode = int(mt_uniform(a, 4u, lane)) + 1;  // "ACGU"[r]
    const int e = st.clo_err[pick];
    bool changed = false;
    if (e == 0) {
        for (int k = st.clo_off[pick] + lane; k < st.clo_off[pick + 1]; k += WAVE) {
            const int pos = st.clo_pos[k];
            const int nb = st.clo_par[k] ? 5 - bcode : bcode;
            if (cur[pos] != nb) changed = true;
        }
        changed = __ballot(changed) != 0ull;
    }
    double u = 0.0;
    if (e == 0 && changed) u = mt_canonical(c, lane);
    for (int k = lane; k < 624; k += WAVE) {
        if (a.twisted) gA[k] = mA[k];
        if (c.twisted) gC[k] = mC[k];
    }
    if (changed) {
        uint8_t *prop = st.prop_seq + size_t(w) * st.Nraw;
        for (int k = lane; k < st.Nraw; k += WAVE) prop[k] = cur[k];
        __syncthreads();
        for (int k = st.clo_off[pick] + lane; k < st.clo_off[pick + 1]; k += WAVE)
            prop[st.clo_pos[k]] = uint8_t(st.clo_par[k] ? 5 - bcode : bcode);
    }
    if (lane == 0) {
        gA[624] = uint32_t(a.idx);
        gC[624] = uint32_t(c.idx);
        st.pick[w] = pick;
        st.bcode[w] = bcode;
        st.temp[w] = T;
        st.u[w] = u;
        st.changed[w] = (e != 0) ? 0 : (changed ? 1 : 0);
        if (e != 0) st.err[w] = e;
        if (st.tr_pos) {
            const size_t r = size_t(s) * st.W + w;
            st.tr_pos[r] = st.mut[pick];
            st.tr_base[r] = int8_t(bcode);
            st.tr_temp[r] = T;
        }
    }
}

__global__ void __launch_bounds__(256) accept_kernel(StepArgs st, int s, int nt_tot) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= st.W || st.err[w]) return;
    const bool changed = st.changed[w] == 1;
    int outcome = 2;  // ACCEPT_UNCHANGED
    const double prop = st.prop_score[w];
    if (changed) {
        const double diff = prop - st.cur_score[w];
        st.last_diff[w] = diff;
        const double crit = exp(diff / st.temp[w]);
        if (crit < st.u[w]) {
            outcome = 0;
        } else {
            outcome = (diff > 0) ? 3 : 1;
            st.cur_score[w] = prop;
            const uint8_t *p = st.prop_seq + size_t(w) * st.Nraw;
            uint8_t *c = st.cur_seq + size_t(w) * st.Nraw;
            for (int k = 0; k < st.Nraw; k++) c[k] = p[k];
        }
    }
    st.counters[size_t(w) * 4 + outcome] += 1;
    if (st.tr_pos) {
        const size_t r = size_t(s) * st.W + w;
        st.tr_outcome[r] = outcome;
        st.tr_prop[r] = changed ? prop : __builtin_nan("");
        st.tr_cur[r] = st.cur_score[w];
        st.tr_u[r] = changed ? st.u[w] : __builtin_nan("");
        if (!changed && st.tr_terms)
            for (int k = 0; k < nt_tot; k++) st.tr_terms[r * nt_tot + k] = __builtin_nan("");
    }
}

}  // namespace

// ---------------------------------------------------------------- host launchers
size_t lds_bytes(const KArgs &ka, bool /*unused*/, int nt) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    const size_t C = size_t(ka.cells);
    const size_t NP = size_t(ka.Nmax) + 2;
    return 3 * al(C * 4) + al(C) + al(2 * nt * 4 + 16) + al(CT_SIZE * 4) + al(size_t(896 + 2 * MAX_SPECIAL_HP + ka.Nmax + 1) * 4) + al(NP * 4) + al(16 * 4) +
           al(size_t(ka.n_variants) * 8) + al(16) + 8 * al(NP) + al(8 * NP);
}

constexpr int NT_DEFAULT = 512;

hipError_t launch_score_m(const KArgs &ka, const uint8_t *seqs, int W, double *scores, double *terms,
                          float *dG, const int *mask, hipStream_t stream) {
    const size_t lds = lds_bytes(ka, true, NT_DEFAULT);
    auto k = score_kernel<NT_DEFAULT>;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(k, dim3(W), dim3(NT_DEFAULT), lds, stream, ka, ka.X, seqs, W, scores, terms, dG, mask);
    return hipGetLastError();
}

hipError_t launch_score(const KArgs &ka, bool, const uint8_t *seqs, int W, double *scores,
                        double *terms, float *dG, hipStream_t stream) {
    return launch_score_m(ka, seqs, W, scores, terms, dG, nullptr, stream);
}

hipError_t launch_steps(const KArgs &ka, bool, const StepArgs &st, hipStream_t stream) {
    const int nt_tot = ka.n_terms * ka.n_ctx_eff;
    for (int s = 0; s < st.nsteps; s++) {
        hipLaunchKernelGGL(propose_kernel, dim3(st.W), dim3(64), 0, stream, st, st.step0 + s, s);
        double *tv = st.tr_terms ? st.tr_terms + size_t(s) * st.W * nt_tot : nullptr;
        hipError_t e = launch_score_m(ka, st.prop_seq, st.W, st.prop_score, tv, nullptr, st.changed, stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(accept_kernel, dim3((st.W + 255) / 256), dim3(256), 0, stream, st, s, nt_tot);
    }
    return hipGetLastError();
}

}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps(unsigned long long *out, int reset) {  // [16][16]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps), sizeof(adx::g_stamps)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
