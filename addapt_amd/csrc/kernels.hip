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

namespace {

constexpr int WAVE = 64;

__device__ __constant__ int8_t PAIR_D[5][5] = {{0, 0, 0, 0, 0},
                                               {0, 0, 0, 0, 5},
                                               {0, 0, 0, 1, 0},
                                               {0, 0, 2, 0, 3},
                                               {0, 6, 0, 4, 0}};
__device__ __constant__ int8_t RTYPE_D[8] = {0, 2, 1, 4, 3, 6, 5, 7};

__device__ __forceinline__ int ptype(int a, int b) { return PAIR_D[a][b]; }

// index of the first cell of diagonal dd (cells with j - i = dd >= 4)
__device__ __forceinline__ int off(int dd, int N) { return ((dd - 4) * (2 * N - 3 - dd)) >> 1; }

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}

// LDS carve-out for one workgroup (see lds_bytes()).
struct Lds {
    float *qb, *qm, *qm1, *qbm;
    float *scrA, *scrB, *q5;
    float *misc;       // [0] = q5 partial
    double *G;         // per-variant ensemble energies
    uint8_t *S, *up, *dn, *ptn, *enc, *flg, *mat;
    uint8_t *lists;    // plist[2] then pinv[2], NP bytes each
    int np;
    int *pcount;       // [2]
    uint8_t *raw;      // proposal / scored sequence (Nraw)
    uint32_t *rng;     // aliased onto the tables: 2 * MT_WORDS
    double *dscr;      // scratch doubles (median etc.)
};

template <int NT>
__device__ Lds carve(char *base, const KArgs &ka, bool qbm) {
    Lds L;
    const int C = ka.cells;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        char *p = base + o;
        o += (bytes + 15) & ~size_t(15);
        return p;
    };
    const size_t tbytes = size_t(C) * 4 * (qbm ? 4 : 3);
    char *tb = take(tbytes > 2 * MT_WORDS * 4 ? tbytes : 2 * MT_WORDS * 4);
    L.qb = reinterpret_cast<float *>(tb);
    L.qm = L.qb + C;
    L.qm1 = L.qm + C;
    L.qbm = qbm ? L.qm1 + C : nullptr;
    L.rng = reinterpret_cast<uint32_t *>(tb);
    L.scrA = reinterpret_cast<float *>(take(NT * 4));
    L.scrB = reinterpret_cast<float *>(take(NT * 4));
    const int NP = ka.Nmax + 2;
    L.q5 = reinterpret_cast<float *>(take(NP * 4));
    L.misc = reinterpret_cast<float *>(take(16 * 4));
    L.G = reinterpret_cast<double *>(take(MAX_VARIANTS * 8));
    L.dscr = reinterpret_cast<double *>(take(16 * 8));
    L.pcount = reinterpret_cast<int *>(take(4 * 4));
    L.S = reinterpret_cast<uint8_t *>(take(NP));
    L.up = reinterpret_cast<uint8_t *>(take(NP));
    L.dn = reinterpret_cast<uint8_t *>(take(NP));
    L.ptn = reinterpret_cast<uint8_t *>(take(NP));
    L.enc = reinterpret_cast<uint8_t *>(take(NP));
    L.flg = reinterpret_cast<uint8_t *>(take(NP));
    L.mat = reinterpret_cast<uint8_t *>(take(NP));
    L.np = NP;
    L.lists = reinterpret_cast<uint8_t *>(take(4 * NP));
    L.raw = reinterpret_cast<uint8_t *>(take(NP));
    return L;
}

__device__ __forceinline__ uint8_t *plist(const Lds &L, int b) { return L.lists + b * L.np; }
__device__ __forceinline__ uint8_t *pinv(const Lds &L, int b) { return L.lists + (2 + b) * L.np; }

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

// wave 0: compact the pairable cells of diagonal dd into buffer b
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
// Returns the ensemble free energy (kcal/mol, double) of variant v folded on
// the raw sequence `raw` (codes, Nraw); all threads of the block must call.
template <int NT, bool QBM>
__device__ double pf_inside(const KArgs &ka, int v, const uint8_t *raw, const Lds &L) {
    constexpr int NW = NT / WAVE;
    const DevVariant V = ka.variants[v];
    const int N = V.N;
    const DevTables &T = *ka.T;
    const DevScaled &X = *ka.X;
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);

    // ---- per-variant setup: sequence, constraint arrays, motif sites
    const uint8_t *cons = ka.cons + V.cons_off;
    const int np = N + 2;
    const uint8_t *bef = nullptr, *aft = nullptr;
    int blen = 0, alen = 0;
    if (V.ctx >= 0) {
        bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
        blen = ka.ctx_off[4 * V.ctx + 1];
        aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
        alen = ka.ctx_off[4 * V.ctx + 3];
    }
    for (int k = tid; k < np; k += NT) {
        uint8_t s = 0;
        if (k >= 1 && k <= N) {
            const int p = k - 1;
            if (p < blen) s = bef[p];
            else if (p < blen + ka.Nraw) s = raw[p - blen];
            else s = aft[p - blen - ka.Nraw];
        }
        L.S[k] = s;
        L.up[k] = cons[k];
        L.dn[k] = cons[np + k];
        L.ptn[k] = cons[2 * np + k];
        L.enc[k] = cons[3 * np + k];
        L.flg[k] = cons[4 * np + k];
        L.mat[k] = 0;
    }
    __syncthreads();
    if (tid == 0) {
        // ViennaRNA's S1 wrap-around (only reaches values that are never used)
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
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
    if (tid < 4) {
        if (tid == 0) L.q5[0] = 1.0f;
    }
    __syncthreads();
    if (tid == 0) {
        for (int j = 1; j <= 3 && j <= N; j++) L.q5[j] = (L.up[j] >= 1) ? L.q5[j - 1] * X.sig[1] : 0.f;
    }
    if (wid == 0 && N - 1 >= 4) build_plist(L, N, 4, 0, lane);
    __syncthreads();

    const float sig1 = X.sig[1];
    const float mlbase_sig = X.mlbase_sig;

    for (int d = 4; d <= N; ++d) {
        const int cur = d & 1;
        const int db = d - 1;
        const bool jobA = d <= N - 1;
        const bool jobB = db >= 4 && db <= N - 6;
        const int cp = jobA ? L.pcount[cur] : 0;
        const int gA = (cp + WAVE - 1) / WAVE;
        const int slA = gA ? NW / gA : 0;
        const int cb = jobB ? N - db : 0;
        const int gB = (cb + WAVE - 1) / WAVE;
        const int slB = gB ? NW / gB : 0;

        // ============================== phase A
        if (cp > 0 && wid < gA * slA) {
            const int ch = wid % gA, sl = wid / gA;
            const int r = ch * WAVE + lane;
            const bool active = r < cp;
            const int i = plist(L, cur)[active ? r : 0];
            const int j = i + d;
            const int si = L.S[i], sj = L.S[j];
            const int type = ptype(si, sj);
            const int si1 = L.S[i + 1], sj1 = L.S[j - 1];
            const int A_ = L.up[i + 1], B_ = L.dn[j - 1];
            const float mm1n_ij = T.mm1n[type][si1][sj1];
            const float mm23_ij = T.mm23[type][si1][sj1];
            const float tau_ij = T.termAU[type];
            float accS = 0.f, accG = 0.f, accM = 0.f;
            const int nInt = (d >= 6) ? X.ncnt[d - 6 < 30 ? d - 6 : 30] : 0;
            int t = sl;
            for (; t < nInt; t += slA) {
                const TermDesc e = X.terms[t];
                const int n1 = e.n1, n2 = e.n2;
                const int base = off(d - 2 - e.u, N);
                const int p = i + 1 + n1, q = j - 1 - n2;
                const int idx = base + p - 1;
                const bool ok = (n1 <= A_) && (n2 <= B_);
                const float fo = ok ? e.f : 0.f;
                if (e.kind == K_GENERIC) {
                    float vq;
                    if constexpr (QBM) {
                        vq = L.qbm[idx];
                    } else {
                        const int t2 = RTYPE_D[ptype(L.S[p], L.S[q])];
                        vq = L.qb[idx] * T.mmI[t2][L.S[q + 1]][L.S[p - 1]];
                    }
                    accG = fmaf(vq, fo, accG);
                } else {
                    const float vq = L.qb[idx];
                    const int sp = L.S[p], sq = L.S[q];
                    const int type2 = ptype(sq, sp);
                    float fac;
                    switch (e.kind) {
                    case K_STACK:
                    case K_BULGE1: fac = T.stack[type][type2]; break;
                    case K_BULGE: fac = tau_ij * T.termAU[type2]; break;
                    case K_I11: fac = T.int11[type][type2][si1][sj1]; break;
                    case K_I21: fac = T.int21[type][type2][si1][L.S[q + 1]][sj1]; break;
                    case K_I12: fac = T.int21[type2][type][L.S[q + 1]][si1][L.S[p - 1]]; break;
                    case K_I22: fac = T.int22[type][type2][si1][L.S[p - 1]][L.S[q + 1]][sj1]; break;
                    case K_I23: fac = mm23_ij * T.mm23[type2][L.S[q + 1]][L.S[p - 1]]; break;
                    default: /* K_1N */ fac = mm1n_ij * T.mm1n[type2][L.S[q + 1]][L.S[p - 1]]; break;
                    }
                    accS = fmaf(vq * fac, fo, accS);
                }
            }
            // multiloop closed by (i,j): k = i + tp, tp in [6, d-5]
            const int nML = d - 10;
            for (int m = t - nInt; m < nML; m += slA) {
                const int tp = m + 6;
                const int idx1 = off(tp - 2, N) + i;           // (i+1, i+tp-1)
                const int idx2 = off(d - 1 - tp, N) + i + tp - 1;  // (i+tp, j-1)
                accM = fmaf(L.qm[idx1], L.qm1[idx2], accM);
            }
            const float mmI_ij = T.mmI[type][si1][sj1];
            const float mlc_ij = X.mlclosing * T.mlstem[RTYPE_D[type]][sj1][si1];
            float part = accS + accG * mmI_ij + accM * mlc_ij;
            L.scrA[(sl * gA + ch) * WAVE + lane] = part;
        }
        if (cb > 0 && wid < gB * slB) {
            const int ch = wid % gB, sl = wid / gB;
            const int r = ch * WAVE + lane;
            const bool active = r < cb;
            const int i = (active ? r : 0) + 1;
            const int upi = L.up[i];
            float acc = 0.f;
            int t = sl;
            const int tmax = db - 4;
            for (; t <= tmax && t < 5; t += slB) {
                const float q1 = L.qm1[off(db - t, N) + i + t - 1];
                const float pre = (t <= upi) ? X.pwml[t] : 0.f;
                acc = fmaf(pre, q1, acc);
            }
            for (; t <= tmax; t += slB) {
                const float q1 = L.qm1[off(db - t, N) + i + t - 1];
                const float pre = ((t <= upi) ? X.pwml[t] : 0.f) + L.qm[off(t - 1, N) + i - 1];
                acc = fmaf(pre, q1, acc);
            }
            L.scrB[(sl * gB + ch) * WAVE + lane] = acc;
        }
        if (wid == NW - 1) {
            // q5[j], j = d: sum_k q5[k-1] qb[k][j] ext(k,j)
            const int j = d;
            float acc = 0.f;
            for (int k = 1 + lane; k <= j - 4; k += WAVE) {
                const float vq = L.qb[off(j - k, N) + k - 1];
                const int type = ptype(L.S[k], L.S[j]);
                const int c5 = (k > 1) ? L.S[k - 1] : 5;
                const int c3 = (j < N) ? L.S[j + 1] : 5;
                acc = fmaf(L.q5[k - 1] * vq, T.ext[type][c5][c3], acc);
            }
            acc = wave_sum(acc);
            if (lane == 0) L.misc[0] = acc;
        }
        __syncthreads();

        // ============================== phase B
        const int cd = jobA ? N - d : 0;
        const int nitems = cd + cb + 1;
        for (int w = tid; w < nitems; w += NT) {
            if (w < cd) {
                const int i = w + 1, j = i + d;
                const int idx = off(d, N) + i - 1;
                const int r = pinv(L, cur)[i];
                const int si = L.S[i], sj = L.S[j];
                const int type = ptype(si, sj);
                float qbv = 0.f;
                if (r != 0xFF) {
                    const int ch = r / WAVE, ln = r % WAVE;
                    for (int sl = 0; sl < slA; sl++) qbv += L.scrA[(sl * gA + ch) * WAVE + ln];
                    const int u = d - 1;
                    if (L.up[i + 1] >= u) {
                        float hpv = -1.f;
                        if (u == 3 || u == 4 || u == 6) {
                            const uint32_t key = hp_key(L.S, i, u + 2);
                            for (int k = 0; k < X.n_special; k++)
                                if (X.sp_key[k] == key) { hpv = X.sp_val[k]; break; }
                        }
                        if (hpv < 0.f)
                            hpv = X.hp[u] * ((u == 3) ? T.termAU[type] : T.mmH[type][L.S[i + 1]][L.S[j - 1]]);
                        qbv += hpv;
                    }
                    if (L.mat[i] && d == X.motif_len - 1) qbv += X.motif_extra;
                }
                L.qb[idx] = qbv;
                if constexpr (QBM) {
                    L.qbm[idx] = qbv * T.mmI[RTYPE_D[type]][L.S[j + 1]][L.S[i - 1]];
                }
                if (d <= N - 6) {
                    float q1 = qbv * T.mlstem[type][L.S[i - 1]][L.S[j + 1]];
                    if (d >= 5 && L.up[j] >= 1) q1 = fmaf(L.qm1[off(d - 1, N) + i - 1], mlbase_sig, q1);
                    L.qm1[idx] = q1;
                }
            } else if (w < cd + cb) {
                const int r = w - cd;
                const int i = r + 1;
                const int ch = r / WAVE, ln = r % WAVE;
                float s = 0.f;
                for (int sl = 0; sl < slB; sl++) s += L.scrB[(sl * gB + ch) * WAVE + ln];
                L.qm[off(db, N) + i - 1] = s;
            } else {
                L.q5[d] = ((L.up[d] >= 1) ? L.q5[d - 1] * sig1 : 0.f) + L.misc[0];
            }
        }
        if (wid == 0 && d + 1 <= N - 1) build_plist(L, N, d + 1, cur ^ 1, lane);
        __syncthreads();
    }
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

template <int NT, bool QBM>
__device__ double score_sequence(const KArgs &ka, const uint8_t *raw, const Lds &L,
                                 float *dG_out, double *terms_out) {
    for (int v = 0; v < ka.n_variants; v++) {
        const double g = pf_inside<NT, QBM>(ka, v, raw, L);
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

template <int NT, bool QBM>
__global__ void __launch_bounds__(NT, 4)
score_kernel(KArgs ka, const uint8_t *seqs, int W, double *scores, double *terms, float *dG) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Lds L = carve<NT>(smem, ka, QBM);
    const int w = blockIdx.x;
    if (w >= W) return;
    for (int k = threadIdx.x; k < ka.Nraw; k += NT) L.raw[k] = seqs[size_t(w) * ka.Nraw + k];
    __syncthreads();
    const int nt = ka.n_terms * ka.n_ctx_eff;
    const double s = score_sequence<NT, QBM>(ka, L.raw, L, dG ? dG + size_t(w) * ka.n_variants : nullptr,
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
// One workgroup = one walker; the walker state that must survive the fold
// (scores, thermostat state, counters) is kept in LDS, not in registers, so
// the PF loop has the whole register file.
template <int NT, bool QBM>
__global__ void __launch_bounds__(NT, 4) step_kernel(KArgs ka, StepArgs st) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Lds L = carve<NT>(smem, ka, QBM);
    const int w = blockIdx.x;
    if (w >= st.W) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);
    const int Nraw = ka.Nraw;
    const int nt_tot = ka.n_terms * ka.n_ctx_eff;
    uint8_t *cur = st.cur_seq + size_t(w) * Nraw;
    uint32_t *gA = st.mtA + size_t(w) * MT_WORDS;
    uint32_t *gC = st.mtC + size_t(w) * MT_WORDS;
    // LDS-resident walker state
    double *sd = L.dscr;                                  // 0 current 1 last_diff 2 autoT 3 u 4 prop 5 median
    int *mi = reinterpret_cast<int *>(L.misc + 4);        // 0 pick 1 base 2 err 3 changed 4 ntrain 5 werr 6..9 counts
    if (tid == 0) {
        sd[0] = st.cur_score[w];
        sd[1] = st.last_diff[w];
        sd[2] = st.auto_T[w];
        mi[4] = st.ntrain[w];
        mi[5] = st.err[w];
        mi[6] = mi[7] = mi[8] = mi[9] = 0;
    }
    __syncthreads();

    for (int s = 0; s < st.nsteps; s++) {
        if (mi[5] != 0) break;
        const long long step = st.step0 + s;
        // ---- thermostat (sampling.cc:59; 309-401)
        double T;
        if (st.thermo_kind == 0) {
            T = st.t_fixed;
        } else if (st.thermo_kind == 1) {
            const int Nc = st.cycle_len;
            T = ((st.t_lo - st.t_hi) / Nc) * double(int(step % Nc)) + st.t_hi;
        } else {
            double *tr = st.train + size_t(w) * st.period;
            const int nt0 = mi[4];
            __syncthreads();
            if (tid == 0) {
                tr[nt0] = sd[1];
                mi[4] = nt0 + 1;
            }
            __syncthreads();
            if (nt0 + 1 >= st.period) {
                // nth_element(n/2): a value whose rank window covers n/2
                const int n = nt0 + 1, k = n / 2;
                if (wid == 0) {
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
                    if (lane == 0) {
                        const double t = med / log(st.target_rate);
                        sd[2] = t > 0.0 ? t : 0.0;
                        mi[4] = 0;
                    }
                }
                __syncthreads();
            }
            T = sd[2];
        }

        // ---- move: wave 0 draws from stream A (and C if the step is scored)
        if (wid == 0) {
            uint32_t *mA = L.rng, *mC = L.rng + MT_WORDS;
            for (int k = lane; k < 624; k += WAVE) {
                mA[k] = gA[k];
                mC[k] = gC[k];
            }
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
            if (lane == 0) {
                gA[624] = uint32_t(a.idx);
                gC[624] = uint32_t(c.idx);
                mi[0] = pick;
                mi[1] = bcode;
                mi[2] = e;
                mi[3] = changed ? 1 : 0;
                sd[3] = u;
            }
        }
        __syncthreads();
        if (mi[2] != 0) {
            if (tid == 0) mi[5] = mi[2];
            break;
        }
        const bool changed = mi[3] != 0;
        double *tv = (st.tr_terms) ? st.tr_terms + (size_t(s) * st.W + w) * nt_tot : nullptr;
        if (changed) {
            const int pick = mi[0], bcode = mi[1];
            for (int k = tid; k < Nraw; k += NT) L.raw[k] = cur[k];
            __syncthreads();
            for (int k = st.clo_off[pick] + tid; k < st.clo_off[pick + 1]; k += NT) {
                const int pos = st.clo_pos[k];
                L.raw[pos] = uint8_t(st.clo_par[k] ? 5 - bcode : bcode);
            }
            __syncthreads();
            const double sc = score_sequence<NT, QBM>(ka, L.raw, L, nullptr, tv);
            if (tid == 0) {
                const double diff = sc - sd[0];
                sd[1] = diff;
                sd[4] = sc;
                const double crit = exp(diff / T);
                int outcome;
                if (crit < sd[3]) {
                    outcome = 0;
                } else {
                    outcome = (diff > 0) ? 3 : 1;
                    sd[0] = sc;
                }
                mi[3] = 2 + outcome;  // 2 REJECT, 3 WORSENED, 5 IMPROVED
            }
            __syncthreads();
            if (mi[3] != 2)
                for (int k = tid; k < Nraw; k += NT) cur[k] = L.raw[k];
        } else if (tv && tid == 0) {
            for (int k = 0; k < nt_tot; k++) tv[k] = __builtin_nan("");
        }
        if (tid == 0) {
            const int outcome = changed ? mi[3] - 2 : 2;
            mi[6 + outcome]++;
            if (st.tr_pos) {
                const size_t r = size_t(s) * st.W + w;
                st.tr_pos[r] = st.mut[mi[0]];
                st.tr_base[r] = int8_t(mi[1]);
                st.tr_outcome[r] = outcome;
                st.tr_temp[r] = T;
                st.tr_prop[r] = changed ? sd[4] : __builtin_nan("");
                st.tr_cur[r] = sd[0];
                st.tr_u[r] = changed ? sd[3] : __builtin_nan("");
            }
        }
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
        for (int k = 0; k < 4; k++) st.counters[size_t(w) * 4 + k] += mi[6 + k];
        st.cur_score[w] = sd[0];
        st.last_diff[w] = sd[1];
        st.auto_T[w] = sd[2];
        st.ntrain[w] = mi[4];
        st.err[w] = mi[5];
    }
}

}  // namespace

// ---------------------------------------------------------------- host launchers
size_t lds_bytes(const KArgs &ka, bool qbm, int nt) {
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    const size_t C = size_t(ka.cells);
    size_t tb = C * 4 * (qbm ? 4 : 3);
    if (tb < 2 * MT_WORDS * 4) tb = 2 * MT_WORDS * 4;
    const size_t NP = size_t(ka.Nmax) + 2;
    size_t s = al(tb) + 2 * al(nt * 4) + al(NP * 4) + al(16 * 4) + al(MAX_VARIANTS * 8) +
               al(16 * 8) + al(16) + 12 * al(NP);
    return s;
}

constexpr int NT_DEFAULT = 512;

hipError_t launch_score(const KArgs &ka, bool qbm, const uint8_t *seqs, int W, double *scores,
                        double *terms, float *dG, hipStream_t stream) {
    const size_t lds = lds_bytes(ka, qbm, NT_DEFAULT);
    if (qbm) {
        auto k = score_kernel<NT_DEFAULT, true>;
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(W), dim3(NT_DEFAULT), lds, stream, ka, seqs, W, scores, terms, dG);
    } else {
        auto k = score_kernel<NT_DEFAULT, false>;
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(W), dim3(NT_DEFAULT), lds, stream, ka, seqs, W, scores, terms, dG);
    }
    return hipGetLastError();
}

hipError_t launch_steps(const KArgs &ka, bool qbm, const StepArgs &st, hipStream_t stream) {
    const size_t lds = lds_bytes(ka, qbm, NT_DEFAULT);
    if (qbm) {
        auto k = step_kernel<NT_DEFAULT, true>;
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(st.W), dim3(NT_DEFAULT), lds, stream, ka, st);
    } else {
        auto k = step_kernel<NT_DEFAULT, false>;
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(st.W), dim3(NT_DEFAULT), lds, stream, ka, st);
    }
    return hipGetLastError();
}

}  // namespace adx
