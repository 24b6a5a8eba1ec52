// gfx950 minimum-free-energy fold, four folds per cell: the apo / holo folds
// of the free AND the constrained macrostate of one context advance together
// (uint2 per cell: .x = free apo|holo, .y = constrained apo|holo, 16-bit halves
// as in mfe_cells.hip).  Same recursion and tables as mfe_cells.hip /
// kernels.hip score_kernel<MinPlus16> (oracle/fold.c orc_mfe_energy); the
// mapping changes:
//
//   * one 1024-thread workgroup (16 waves) per walker and one walker per CU:
//     the four folds' tables take ~112 KB of LDS at N = 100;
//   * every LDS read of a DP value is a ds_read_b64 that serves four folds at
//     the LDS cost of one, and every sequence-dependent loop correction (the
//     cc / ct lookups, the per-loop-size energies) is read once for the four;
//   * lanes = cells of one anti-diagonal, the interior-loop shapes in 14
//     generated blocks (mfe_quad_blocks.inc) on waves 0-13, the multiloop (qm)
//     rows on waves 15 / 14, finalize and q5 on waves 14 / 13 / 12; one barrier
//     per diagonal.  Phases per step d exactly as mfe_cells.hip (F, B, M, Q).
//
// The constraint-dependent parts (pairable cells, unpaired runs, the ligand
// motif's sites, the unpaired prefixes of the multiloop and exterior loops)
// are evaluated per word; everything else is shared.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev_types.hpp"
#include "fold_common.hpp"

namespace adx {

#ifdef ADX_STAMP
// Diagnostic build only: per-wave cycle sums of the per-step phases (s_memtime),
// read back through adx_debug_stamps_quad().  Never in the product.
__device__ unsigned long long g_stamps_q[16][16];
#define QSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define QSTAMP(k) do { } while (0)
#endif

namespace {

using u32 = uint32_t;
constexpr u32 INF16 = 0x7FFF7FFFu;
constexpr u32 MARK16 = 0x7FFE7FFEu;   // non-pairable cell of a fold pair (setup value; a finished cell never takes it)
constexpr int QWV = 16;                // waves per walker
constexpr int QNB = 14;                // interior-loop blocks (waves 0-13)

__device__ __forceinline__ s16x2 sv(u32 x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ u32 su(s16x2 x) { return __builtin_bit_cast(u32, x); }
__device__ __forceinline__ u32 pmin(u32 a, u32 b) { return su(__builtin_elementwise_min(sv(a), sv(b))); }
__device__ __forceinline__ u32 padd(u32 a, u32 b) { return su(__builtin_elementwise_add_sat(sv(a), sv(b))); }
__device__ __forceinline__ u32 pfin(u32 u) {   // halves in [0x4000, 0x7FFF] -> 0x7FFF
    const u32 imp = (u & ~(u >> 1)) & 0x40004000u;
    return u | ((imp >> 14) * 0x7FFFu);
}
__device__ __forceinline__ uint2 qmin(uint2 a, uint2 b) { return make_uint2(pmin(a.x, b.x), pmin(a.y, b.y)); }
__device__ __forceinline__ uint2 qadd(uint2 a, u32 c) { return make_uint2(padd(a.x, c), padd(a.y, c)); }
__device__ __forceinline__ uint2 qadd2(uint2 a, uint2 b) { return make_uint2(padd(a.x, b.x), padd(a.y, b.y)); }
__device__ __forceinline__ uint2 qfin(uint2 a) { return make_uint2(pfin(a.x), pfin(a.y)); }
__device__ __forceinline__ uint2 qinf() { return make_uint2(INF16, INF16); }

template <int CTRL, int ROWS>
__device__ __forceinline__ u32 dpp_min(u32 v) {
    const int moved = __builtin_amdgcn_update_dpp(int(INF16), int(v), CTRL, ROWS, 0xf, false);
    return pmin(v, u32(moved));
}
__device__ __forceinline__ u32 wave_min(u32 v) {   // full-wave min, result uniform
    v = dpp_min<0xb1, 0xf>(v);
    v = dpp_min<0x4e, 0xf>(v);
    v = dpp_min<0x114, 0xf>(v);
    v = dpp_min<0x118, 0xf>(v);
    v = dpp_min<0x142, 0xa>(v);
    v = dpp_min<0x143, 0xc>(v);
    return u32(__builtin_amdgcn_readlane(int(v), 63));
}

// ---------------------------------------------------------------- LDS carve
struct QL {
    uint2 *qbm, *qm, *qm1;   // cell tables (fold_common.hpp indexing)
    uint2 *mla;              // [2][np]
    uint2 *q5;               // [np]
    uint2 *part;             // [2][14][64]: interior-loop partial minima, by step parity
    u32 *ct, *dt, *pw;
    uint4 *ku;               // [32][2] per loop size (mfe_cells.hip CL::ku)
    uint2 *mpart;            // [2][64]: wave 14's half of a split qm row (split, unpaired)
    int *mflag;              // step whose half is in mpart
    double *G;
    uint8_t *cc, *S, *raw;
    uint8_t *up[2], *dn[2], *ptn[2], *enc[2], *flg[2], *mat[2];   // per constraint set (free, constrained)
    int np;
};
constexpr size_t al16(size_t b) { return (b + 15) & ~size_t(15); }
constexpr int MFQ_MAXVAR = 32;
template <int NM>
struct QLay {
    static constexpr int NP = NM + 2;
    static constexpr size_t C = size_t(NM - 4) * (NM - 3) / 2;
    static constexpr size_t QBM = 0;
    static constexpr size_t QM = QBM + al16(C * 8);
    static constexpr size_t QM1 = QM + al16(C * 8);
    static constexpr size_t MLA = QM1 + al16(C * 8);
    static constexpr size_t Q5 = MLA + al16(2 * NP * 8);
    static constexpr size_t PART = Q5 + al16(NP * 8);
    static constexpr size_t CT = PART + al16(2 * QNB * 64 * 8);
    static constexpr size_t DT = CT + al16(CT_SIZE * 4);
    static constexpr size_t PW = DT + al16(size_t(DT_HP) * 4);
    static constexpr size_t KU = PW + al16(size_t(NM + 1) * 4);
    static constexpr size_t MP = KU + 32 * 32;
    static constexpr size_t G = MP + 2 * 64 * 8 + 16;
    static constexpr size_t CC = G + al16(MFQ_MAXVAR * 8);
    static constexpr size_t BY = CC + al16(C);   // 14 byte arrays of NP
    static constexpr size_t BYTES = BY + al16(14 * NP);
    __device__ static QL carve(char *b) {
        QL l;
        l.qbm = reinterpret_cast<uint2 *>(b + QBM);
        l.qm = reinterpret_cast<uint2 *>(b + QM);
        l.qm1 = reinterpret_cast<uint2 *>(b + QM1);
        l.mla = reinterpret_cast<uint2 *>(b + MLA);
        l.q5 = reinterpret_cast<uint2 *>(b + Q5);
        l.part = reinterpret_cast<uint2 *>(b + PART);
        l.ct = reinterpret_cast<u32 *>(b + CT);
        l.dt = reinterpret_cast<u32 *>(b + DT);
        l.pw = reinterpret_cast<u32 *>(b + PW);
        l.ku = reinterpret_cast<uint4 *>(b + KU);
        l.mpart = reinterpret_cast<uint2 *>(b + MP);
        l.mflag = reinterpret_cast<int *>(b + MP + 2 * 64 * 8);
        l.G = reinterpret_cast<double *>(b + G);
        l.cc = reinterpret_cast<uint8_t *>(b + CC);
        uint8_t *y = reinterpret_cast<uint8_t *>(b + BY);
        l.S = y;
        l.raw = y + NP;
        for (int g = 0; g < 2; g++) {
            uint8_t *z = y + (2 + 6 * g) * NP;
            l.up[g] = z;
            l.dn[g] = z + NP;
            l.ptn[g] = z + 2 * NP;
            l.enc[g] = z + 3 * NP;
            l.flg[g] = z + 4 * NP;
            l.mat[g] = z + 5 * NP;
        }
        l.np = NP;
        return l;
    }
};

// LDS byte address of an LDS object (the inline-asm batches address LDS directly)
typedef __attribute__((address_space(3))) char lds_char;
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T *p) {
    return uint32_t(uintptr_t((lds_char *)(p)));   // generic -> LDS address space
}

__device__ __forceinline__ bool allowed(const QL &L, int g, int i, int j) {   // kernels.hip allowed()
    const int fi = L.flg[g][i], fj = L.flg[g][j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[g][i], pj = L.ptn[g][j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[g][i] == L.enc[g][j];
}

// ---------------------------------------------------------------- interior-loop shapes
struct QUni {
    uint32_t aq, ac, aku;        // LDS byte addresses of qbm, cc, ku (inline-asm batches)
    const uint2 *qbm;
    const uint8_t *cc;
    const u32 *ct;
    const uint4 *ku;
    const u32 *gct, *il, *nin;   // HBM (runtime path only)
    u32 fs1;
    int d, N, umax;
    __device__ __forceinline__ int offu(int u) const { return off(d - 2 - u, N); }
};
struct QCell {
    int i, ty8;
    int A0, B0, A1, B1;          // unpaired runs up[i+1] / dn[j-1] of the two constraint sets
    u32 m23f, t11, t12, t21, t22;
};
struct QAcc {
    uint2 s, g0, g1, b, n;
};

#define MFQ_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
// one loop size's LDS reads first, then its arithmetic (0x100 = DS read, 0x2 = VALU)
#ifndef MFQ_NO_GROUP_ORDER
#define MFQ_GROUP_ORDER(n) do { __builtin_amdgcn_sched_group_barrier(0x100, n, 0); __builtin_amdgcn_sched_group_barrier(0x2, 1000, 0); } while (0)
#else
#define MFQ_GROUP_ORDER(n) do { } while (0)
#endif
// a DP value read through its own address register: adjacent cells would
// otherwise merge into ds_read2_b64 (8 LDS cycles against 2 x 2)
__device__ __forceinline__ uint2 ldq(const uint2 *base, int idx) {
#ifndef MFQ_ALLOW_READ2
    asm("" : "+v"(idx));   // opaque, not volatile (no scheduling barrier)
#endif
    return base[idx];
}
#ifndef MFQ_MCH
#define MFQ_MCH 8   // qm split points per load batch
#endif
#include "mfe_quad_blocks.inc"

// Lane-sets with constrained cells (a run shorter than the span's loops): the
// same shapes one at a time, runtime offsets, per-word masks.
__device__ void mfq_block_masked(int b, const QUni &U, const QCell &C, QAcc &a) {
    for (int t = 0; t < int(sizeof(MFQ_BLK_U[0])); t++) {
        const int u = MFQ_BLK_U[b][t];
        if (u < 0 || u > U.umax) return;
        const int o = U.offu(u) + C.i;
        const uint2 *q = U.qbm + o;
        const uint8_t *k = U.cc + o;
        const u32 ilu = U.il[u];
        for (int u1 = 0; u1 <= u; u1++) {
            const int u2 = u - u1;
            const bool ok0 = u1 <= C.A0 && u2 <= C.B0, ok1 = u1 <= C.A1 && u2 <= C.B1;
            if (!ok0 && !ok1) continue;
            uint2 v = q[u1];
            v.x = ok0 ? v.x : INF16;
            v.y = ok1 ? v.y : INF16;
            const int c2 = k[u1];
            const int nl = u1 > u2 ? u1 : u2, ns = u1 > u2 ? u2 : u1;
            const u32 inv = U.ct[CT_INVMM + c2];
            if (nl == 0 || (nl == 1 && ns == 0)) {
                u32 e = padd(inv, U.ct[CT_STK + C.ty8 + ((c2 * 41) >> 10)]);
                if (nl == 1) e = padd(e, U.fs1);
                a.s = qmin(a.s, qadd(v, e));
            } else if (ns == 0) {
                a.b = qmin(a.b, qadd(v, padd(U.ct[CT_BUL + c2], U.gct[CT_FB + nl])));
            } else if (ns == 1 && nl >= 3) {
                a.n = qmin(a.n, qadd(v, padd(U.ct[CT_ONEN + c2], U.gct[CT_F1N + nl])));
            } else if (ns == 1) {
                const u32 tv = (nl == 1) ? C.t11 : (u1 == 1 ? C.t12 : C.t21);
                a.s = qmin(a.s, qadd(v, padd(inv, tv)));
            } else if (ns == 2 && nl == 2) {
                a.s = qmin(a.s, qadd(v, padd(inv, C.t22)));
            } else if (ns == 2 && nl == 3) {
                a.s = qmin(a.s, qadd(v, padd(padd(inv, U.ct[CT_M23O + c2]), C.m23f)));
            } else {
                a.g0 = qmin(a.g0, qadd(v, ilu + U.nin[u1 > u2 ? u1 - u2 : u2 - u1]));
            }
        }
    }
}

// ---------------------------------------------------------------- one quad group
struct IncQ {
    const u32 *src[2];   // per word: the group's tables of the current sequence (null: fold all)
    u32 *dst[2];         // per word: where this fold's tables go (null: nowhere)
    int m_lo, m_hi;
};

__device__ __forceinline__ int lanesets(int n) { return (n + 63) >> 6; }

// groups ga (word x) and gb (word y) share the context (sequence); gb == ga folds one group twice
template <int NT, int NM>
__device__ __forceinline__ void mfq_fold(const KArgs &ka, const DevScaled *__restrict__ XS,
                                         const DevTables *__restrict__ TT, int ga, int gb, const QL &L, uint2 &z,
                                         bool &bad, const IncQ &inc) {
    static_assert(NT == QWV * WAVE, "16 waves");
    const int vsg[2][2] = {{ka.groups2[2 * ga], ka.groups2[2 * ga + 1]}, {ka.groups2[2 * gb], ka.groups2[2 * gb + 1]}};
    const DevVariant V = ka.variants[vsg[0][0]];
    const int N = uni(V.N);
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);
    const int NP = L.np;
    const u32 *gct = reinterpret_cast<const u32 *>(XS->ctab);
    const bool incr = inc.src[0] != nullptr;
    const int m_lo = uni(inc.m_lo), m_hi = uni(inc.m_hi);
    auto clo = [&](int dd) { return incr ? max(1, m_lo - 1 - dd) : 1; };
    auto chi = [&](int dd) { return incr ? min(N - dd, m_hi + 1) : N - dd; };
    auto qlo = [&](int s) { return incr ? max(1, m_lo - 2 - s) : 1; };
    auto qhi = [&](int s) { return incr ? min(N - s, m_hi + 2) : N - s; };

    // ---- sequence, the two constraint sets, motif sites
    const int np = N + 2;
    const uint8_t *bef = nullptr, *aft = nullptr;
    int blen = 0;
    if (V.ctx >= 0) {
        bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
        blen = ka.ctx_off[4 * V.ctx + 1];
        aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
    }
    const uint8_t *cons[2] = {ka.cons + ka.variants[vsg[0][0]].cons_off, ka.cons + ka.variants[vsg[1][0]].cons_off};
    bool constrained = false;
    for (int k = tid; k < np; k += NT) {
        uint8_t s = 0;
        if (k >= 1 && k <= N) {
            const int pp = k - 1;
            if (pp < blen) s = bef[pp];
            else if (pp < blen + ka.Nraw) s = L.raw[pp - blen];
            else s = aft[pp - blen - ka.Nraw];
        }
        L.S[k] = s;
#pragma unroll
        for (int g = 0; g < 2; g++) {
            const uint8_t f = cons[g][4 * np + k], pt = cons[g][2 * np + k];
            L.up[g][k] = cons[g][k];
            L.dn[g][k] = cons[g][np + k];
            L.ptn[g][k] = pt;
            L.enc[g][k] = cons[g][3 * np + k];
            L.flg[g][k] = f;
            L.mat[g][k] = 0;
            if (k >= 1 && k <= N && (f || pt)) constrained = true;
        }
    }
    for (int k = tid; k < 2 * NP; k += NT) L.mla[k] = qinf();
    if (tid == 0) *L.mflag = 0;
    {
        const int C = ((N - 4) * (N - 3)) >> 1;
        for (int k = tid; k < C; k += NT) L.qm[k] = qinf();
    }
    constrained = __syncthreads_or(constrained);
    if (tid == 0) {
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
    }
    // holo halves: per word, per 16-bit half (0x7FFF = no-op for min)
    u32 mextra[2];
    bool anym = false;
    const u32 mx = __float_as_uint(XS->motif_extra);
#pragma unroll
    for (int g = 0; g < 2; g++) {
        const bool m0 = ka.variants[vsg[g][0]].motif != 0, m1 = ka.variants[vsg[g][1]].motif != 0;
        mextra[g] = (m0 ? (mx & 0xFFFFu) : 0x7FFFu) | (m1 ? (mx & 0xFFFF0000u) : 0x7FFF0000u);
        anym |= m0 || m1;
    }
    const int mL = XS->motif_len;
    if (anym && mL > 0) {
        for (int o = tid + 1; o + mL - 1 <= N; o += NT) {
            bool seq_ok = true;
            for (int k = 0; k < mL && seq_ok; k++)
                if (L.S[o + k] != XS->motif_code[k]) seq_ok = false;
#pragma unroll
            for (int g = 0; g < 2; g++) {
                bool ok = seq_ok;
                for (int k = 0; k < mL && ok; k++) {
                    const int pk = XS->motif_pt[k];
                    if (pk < 0) ok = L.up[g][o + k] >= 1;
                    else if (pk > k) ok = allowed(L, g, o + k, o + pk);
                }
                L.mat[g][o] = ok ? 1 : 0;
            }
        }
    }
    __syncthreads();
    const u32 mlclosing = __float_as_uint(XS->mlclosing);
    const u32 mlbase = __float_as_uint(XS->mlbase_sig);
    const int nsp = XS->n_special < MAX_SPECIAL_HP ? XS->n_special : MAX_SPECIAL_HP;
    if (tid == 0) {
        L.q5[0] = make_uint2(0u, 0u);
        for (int j = 1; j <= 4 && j <= N; j++)
            L.q5[j] = make_uint2(L.up[0][j] >= 1 ? L.q5[j - 1].x : INF16, L.up[1][j] >= 1 ? L.q5[j - 1].y : INF16);
    }
    // ---- per-cell setup: inner-pair code, hairpin (+ motif) energy or the
    // non-pairable mark per word, multiloop-stem energy of pairable cells
    for (int dd = 4 + wid; dd <= N - 1; dd += QWV) {
        const int od = off(dd, N);
        const int u = dd - 1;
        for (int r = lane; r < N - dd; r += WAVE) {
            const int i = r + 1, j = i + dd;
            const int si = L.S[i], sj = L.S[j], sim = L.S[i - 1], sjp = L.S[j + 1];
            const int type = ptype(si, sj);
            u32 qv[2], mv[2];
            if (type != 0) {
                u32 hs = INF16;
                bool special = false;
                if (u == 3 || u == 4 || u == 6) {
                    const uint32_t key = hp_key(L.S, i, u + 2);
                    for (int k = 0; k < nsp; k++)
                        if (XS->sp_key[k] == key) { hs = __float_as_uint(XS->sp_val[k]); special = true; break; }
                }
                if (!special)
                    hs = padd(__float_as_uint(XS->hp[u]), (u == 3) ? L.dt[DT_TAU + type]
                                                                 : L.dt[DT_MMH + type * 25 + L.S[i + 1] * 5 + L.S[j - 1]]);
                const u32 m1 = L.dt[DT_MLS + type * 25 + sim * 5 + sjp];
#pragma unroll
                for (int g = 0; g < 2; g++) {
                    const bool pr = allowed(L, g, i, j);
                    u32 h = (L.up[g][i + 1] >= u) ? hs : INF16;
                    if (dd == mL - 1 && mL > 0 && L.mat[g][i]) h = pmin(h, mextra[g]);
                    qv[g] = pr ? h : MARK16;
                    mv[g] = pr ? m1 : INF16;
                }
            } else {
                qv[0] = qv[1] = MARK16;
                mv[0] = mv[1] = INF16;
            }
            L.qbm[od + r] = make_uint2(qv[0], qv[1]);
            L.qm1[colb(j) + i - 1] = make_uint2(mv[0], mv[1]);
            L.cc[od + r] = static_cast<uint8_t>(rtype(type) * 25 + sjp * 5 + sim);
        }
    }
    __syncthreads();
    // ---- incremental fold: the unchanged cells from the current sequence's tables
    if (incr) {
        const size_t C = size_t(ka.cells);
        const u32 *s0 = inc.src[0], *s1 = inc.src[1];
        for (int dd = 4 + wid; dd <= N - 1; dd += QWV) {
            const int lo = clo(dd), hi = chi(dd), od = off(dd, N);
            for (int r = lane; r < N - dd; r += WAVE) {
                const int i = r + 1, j = i + dd;
                if (i >= lo && i <= hi) continue;
                const int a = od + r, b = rowb(i, N) + dd - 4, c = colb(j) + i - 1;
                L.qbm[a] = make_uint2(s0[a], s1[a]);
                L.qm[b] = make_uint2(s0[C + b], s1[C + b]);
                L.qm1[c] = make_uint2(s0[2 * C + c], s1[2 * C + c]);
            }
        }
        for (int k = tid; k <= m_lo - 2 && k <= N; k += NT) L.q5[k] = make_uint2(s0[3 * C + k], s1[3 * C + k]);
        __syncthreads();
    }

    const DevTables &T = *TT;
    const u32 *T11 = reinterpret_cast<const u32 *>(&T.int11[0][0][0][0]);
    const u32 *T21 = reinterpret_cast<const u32 *>(&T.int21[0][0][0][0][0]);
    const u32 *T22 = reinterpret_cast<const u32 *>(&T.int22[0][0][0][0][0][0]);
    const u32 tauE = gct[CT_FSM + 6];
    const u32 fsm5 = gct[CT_FSM + 5];
    QUni U;
    U.qbm = L.qbm;
    U.cc = L.cc;
    U.ct = L.ct;
    U.ku = L.ku;
    U.aq = lds_addr(L.qbm);
    U.ac = lds_addr(L.cc);
    U.aku = lds_addr(L.ku);
    const uint32_t aqm = lds_addr(L.qm), aqm1 = lds_addr(L.qm1), aqbm = lds_addr(L.qbm), amla = lds_addr(L.mla);
    const uint32_t aSb = lds_addr(L.S), aup0 = lds_addr(L.up[0]), aup1 = lds_addr(L.up[1]), acc0 = lds_addr(L.cc);
    const uint32_t apart = lds_addr(L.part);
    U.gct = gct;
    U.il = reinterpret_cast<const u32 *>(XS->il);
    U.nin = reinterpret_cast<const u32 *>(XS->nin);
    U.fs1 = gct[CT_FSM + 1];
    U.N = N;
    // wave roles besides the interior-loop blocks
    constexpr int WM0 = 15, WM1 = 14;   // qm lane-sets 0 / 1 (2: wave 15 again)
    constexpr int WF0 = 13, WF1 = 12;   // finalize lane-sets 0 / 1
    constexpr int WQ = 11;              // q5

#ifdef ADX_STAMP
    unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    for (int d = 4; d <= N + 1; ++d) {
        QSTAMP(0);
        // ---------------- F: finalize diagonal e = d - 1
        const int e = d - 1;
        if (e >= 4 && e <= N - 1) {
            const int lo = clo(e), hi = chi(e);
            const int Le = lanesets(hi - lo + 1);
            const int fls = wid == WF0 ? 0 : (wid == WF1 ? 1 : 2);
            if (fls < Le) {
                const int i0 = lo + fls * WAVE + lane;
                const bool fvalid = i0 <= hi;
                const int i = fvalid ? i0 : hi;   // every lane reads (the batch below is unconditional)
                {
                    const int j = i + e;
                    const int ce = off(e, N) + i - 1;
                    const int cm = colb(j) + i - 1;
                    const int pbase = (e & 1) * QNB + (Le == 1 ? 0 : fls * (QNB / 2));
                    // every independent read of the finalize in one batch (mfe_quad_blocks.inc)
                    uint2 init, pq, st, ml, pv[QNB];
                    uint32_t si, sj, si1, sj1, u0j, u1j, cce;
                    {
                        const uint32_t aqb = aqbm + uint32_t(ce) * 8u, aq1 = aqm1 + uint32_t(cm) * 8u;
                        const uint32_t aq1p = aqm1 + uint32_t(colb(j - 1) + i - 1) * 8u;
                        const uint32_t aml = amla + uint32_t(((e - 2) & 1) * NP + i + 1) * 8u;
                        const uint32_t aS = aSb + uint32_t(i), aSj = aSb + uint32_t(j);
                        const uint32_t au0 = aup0 + uint32_t(j), au1 = aup1 + uint32_t(j);
                        const uint32_t acc = acc0 + uint32_t(ce);
                        const uint32_t ap = apart + uint32_t(pbase * WAVE + lane) * 8u;
                        asm volatile(
                            "ds_read_b64 %[init], %[aqb]\n"
                            "ds_read_b64 %[pq], %[aq1p]\n"
                            "ds_read_b64 %[st], %[aq1]\n"
                            "ds_read_b64 %[ml], %[aml]\n"
                            "ds_read_u8 %[si], %[aS]\n"
                            "ds_read_u8 %[si1], %[aS] offset:1\n"
                            "ds_read_u8 %[sj], %[aSj]\n"
                            "ds_read_u8 %[sj1], %[aSj1]\n"
                            "ds_read_u8 %[u0j], %[au0]\n"
                            "ds_read_u8 %[u1j], %[au1]\n"
                            "ds_read_u8 %[cce], %[acc]\n"
                            "ds_read_b64 %[p0], %[ap] offset:0\n"
                            "ds_read_b64 %[p1], %[ap] offset:512\n"
                            "ds_read_b64 %[p2], %[ap] offset:1024\n"
                            "ds_read_b64 %[p3], %[ap] offset:1536\n"
                            "ds_read_b64 %[p4], %[ap] offset:2048\n"
                            "ds_read_b64 %[p5], %[ap] offset:2560\n"
                            "ds_read_b64 %[p6], %[ap] offset:3072\n"
                            "ds_read_b64 %[p7], %[ap] offset:3584\n"
                            "ds_read_b64 %[p8], %[ap] offset:4096\n"
                            "ds_read_b64 %[p9], %[ap] offset:4608\n"
                            "ds_read_b64 %[p10], %[ap] offset:5120\n"
                            "ds_read_b64 %[p11], %[ap] offset:5632\n"
                            "ds_read_b64 %[p12], %[ap] offset:6144\n"
                            "ds_read_b64 %[p13], %[ap] offset:6656\n"
                            "s_waitcnt lgkmcnt(0)"
                            : [init] "=&v"(init), [pq] "=&v"(pq), [st] "=&v"(st), [ml] "=&v"(ml), [si] "=&v"(si),
                              [si1] "=&v"(si1), [sj] "=&v"(sj), [sj1] "=&v"(sj1), [u0j] "=&v"(u0j), [u1j] "=&v"(u1j),
                              [cce] "=&v"(cce), [p0] "=&v"(pv[0]), [p1] "=&v"(pv[1]), [p2] "=&v"(pv[2]),
                              [p3] "=&v"(pv[3]), [p4] "=&v"(pv[4]), [p5] "=&v"(pv[5]), [p6] "=&v"(pv[6]),
                              [p7] "=&v"(pv[7]), [p8] "=&v"(pv[8]), [p9] "=&v"(pv[9]), [p10] "=&v"(pv[10]),
                              [p11] "=&v"(pv[11]), [p12] "=&v"(pv[12]), [p13] "=&v"(pv[13])
                            : [aqb] "v"(aqb), [aq1p] "v"(aq1p), [aq1] "v"(aq1), [aml] "v"(aml), [aS] "v"(aS),
                              [aSj] "v"(aSj), [aSj1] "v"(aSj - 1u), [au0] "v"(au0), [au1] "v"(au1), [acc] "v"(acc), [ap] "v"(ap)
                            : "memory");
                    }
                    const uint2 prev = make_uint2((e >= 5 && u0j >= 1) ? padd(pq.x, mlbase) : INF16,
                                                  (e >= 5 && u1j >= 1) ? padd(pq.y, mlbase) : INF16);
                    uint2 f1 = prev;
                    const bool p0 = init.x != MARK16, p1 = init.y != MARK16;
                    if (fvalid && (p0 || p1)) {
                        uint2 c = init;
                        if (e >= 6) {   // no interior loop fits a span below 6
                            const int nsl = Le == 1 ? QNB : QNB / 2;   // the lane-set layout B used at step e
#pragma unroll
                            for (int b = 0; b < QNB; b++) c = (b < nsl) ? qmin(c, pv[b]) : c;
                        }
                        const int ty = ptype(si, sj);
                        const u32 mlcl = padd(mlclosing, L.dt[DT_MLS + rtype(ty) * 25 + sj1 * 5 + si1]);
                        c = qfin(qmin(c, qadd(ml, mlcl)));
                        const uint2 fq = qfin(qadd(c, L.dt[DT_MMI + cce]));
                        L.qbm[ce] = make_uint2(p0 ? fq.x : MARK16, p1 ? fq.y : MARK16);
                        f1 = make_uint2(p0 ? pmin(padd(c.x, st.x), prev.x) : prev.x,
                                        p1 ? pmin(padd(c.y, st.y), prev.y) : prev.y);
                    }
                    if (fvalid) L.qm1[cm] = qfin(f1);
                }
            }
        }
        QSTAMP(1);
        // ---------------- B: interior-loop partials of diagonal d
        if (d <= N - 1 && d >= 6 && wid < QNB) {
            const int lo = clo(d), hi = chi(d);
            const int Lb = lanesets(hi - lo + 1);
            // one lane-set: wave w runs block w; two: wave w runs blocks w % 7 and w % 7 + 7
            // (the halves of one 7-block) on lane-set w / 7
            const int ls = Lb == 1 ? 0 : wid / (QNB / 2);
            const int slot = Lb == 1 ? wid : ls * (QNB / 2) + wid % (QNB / 2);
            int i = lo + ls * WAVE + lane;
            const bool valid = i <= hi;
            if (!valid) i = hi;
            const int j = i + d;
            const uint2 q0 = L.qbm[off(d, N) + i - 1];
            const bool pr = valid && (q0.x != MARK16 || q0.y != MARK16);
            if (ls < Lb && pr) {   // only pairable cells' lanes (fewer lanes in bank-conflicting reads)
                const int umax = d - 6 < 30 ? d - 6 : 30;
                U.d = d;
                U.umax = umax;
                QCell C;
                const int type = ptype(L.S[i], L.S[j]);
                const int si1 = L.S[i + 1], sj1 = L.S[j - 1];
                const int oc = type * 25 + si1 * 5 + sj1;
                C.i = i;
                C.ty8 = type * 8;
                C.A0 = L.up[0][i + 1];
                C.B0 = L.dn[0][j - 1];
                C.A1 = L.up[1][i + 1];
                C.B1 = L.dn[1][j - 1];
                const u32 mmo = L.dt[DT_MMI + oc];
                const u32 tau = type > 2 ? tauE : 0u;
                const u32 mo = padd(L.ct[CT_ONEN + oc], mmo);
                C.m23f = padd(L.ct[CT_M23O + oc], fsm5);
                const int b0 = Lb == 1 ? wid : wid % (QNB / 2);
                const int b1 = Lb == 1 ? -1 : b0 + QNB / 2;
                C.t11 = C.t12 = C.t21 = C.t22 = INF16;
                if (((MFQ_TABLE_BLOCKS >> b0) & 1) || (b1 >= 0 && ((MFQ_TABLE_BLOCKS >> b1) & 1))) {
                    const int ty8 = type * 8;
                    if (umax >= 2) {
                        const int c2 = L.cc[off(d - 4, N) + i + 1];
                        C.t11 = T11[((ty8 + ((c2 * 41) >> 10)) * 5 + si1) * 5 + sj1];
                    }
                    if (umax >= 3) {
                        const int o3 = off(d - 5, N) + i;
                        const int a2 = L.cc[o3 + 1], b2 = L.cc[o3 + 2];
                        const int ta = (a2 * 41) >> 10, tb = (b2 * 41) >> 10;
                        C.t12 = T21[(((ty8 + ta) * 5 + si1) * 5 + (a2 / 5) % 5) * 5 + sj1];
                        C.t21 = T21[(((tb * 8 + type) * 5 + (b2 / 5) % 5) * 5 + si1) * 5 + b2 % 5];
                    }
                    if (umax >= 4) {
                        const int c2 = L.cc[off(d - 6, N) + i + 2];
                        const int t2 = (c2 * 41) >> 10;
                        C.t22 = T22[((((ty8 + t2) * 5 + si1) * 5 + c2 % 5) * 5 + (c2 / 5) % 5) * 5 + sj1];
                    }
                }
                QAcc a{qinf(), qinf(), qinf(), qinf(), qinf()};
                // a word's runs only matter where that word's cell is pairable
                const bool m0 = q0.x != MARK16 && (C.A0 < umax || C.B0 < umax);
                const bool m1 = q0.y != MARK16 && (C.A1 < umax || C.B1 < umax);
                const bool mk = constrained && __ballot(valid && (m0 || m1)) != 0;
                if (mk) {
                    mfq_block_masked(b0, U, C, a);
                    if (b1 >= 0) mfq_block_masked(b1, U, C, a);
                } else {
                    mfq_block(b0, U, C, a);
                    if (b1 >= 0) mfq_block(b1, U, C, a);
                }
                const uint2 acc = qmin(qmin(a.s, qadd(qmin(a.g0, a.g1), mmo)), qmin(qadd(a.b, tau), qadd(a.n, mo)));
                L.part[((d & 1) * QNB + slot) * WAVE + lane] = acc;
            }
        }
        QSTAMP(2);
        // ---------------- M: qm (fML) and mla of span s = d - 2.  Two lane-sets:
        // one per wave (15, 14); one lane-set with a long row: wave 14 folds the
        // upper split points and hands them to wave 15 through LDS (mpart/mflag)
        {
            const int s = d - 2;
            if (s >= 4 && s <= N - 3 && (wid == WM0 || wid == WM1)) {
                const int lo = qlo(s), hi = qhi(s);
                const int Lm = lanesets(hi - lo + 1);
                const int T = s - 4;
                // partial minima of lane-set ls over the split points t in [ta, tb]
                auto mrow = [&](int ls, int ta, int tb, uint2 &split, uint2 &unp, int &i, bool &valid) {
                    i = lo + ls * WAVE + lane;
                    valid = i <= hi;
                    if (!valid) i = hi;
                    const int j = i + s;
                    const uint2 *A1 = L.qm1 + colb(j) + i - 1;   // qm1(i+t, j)
                    const uint2 *R = L.qm + rowb(i, N) - 5;       // qm(i, i+t-1), t >= 5
                    const int up0 = L.up[0][i], up1 = L.up[1][i];
                    const bool umask = __ballot(up0 < tb || up1 < tb) != 0;
                    uint2 sp0 = qinf(), sp1 = qinf(), un0 = qinf(), un1 = qinf();
                    const u32 mlb2 = padd(mlbase, mlbase);
                    if (ta == 0) {   // t = 0..4: the unpaired prefix only (reads past T are in LDS and masked)
                        uint2 av[5];
#pragma unroll
                        for (int k = 0; k < 5; k++) av[k] = A1[k];
                        u32 pwt = 0u;
#pragma unroll
                        for (int k = 0; k < 5; k++) {
                            if (k <= T) {
                                if (k <= up0) un0.x = pmin(un0.x, padd(pwt, av[k].x));
                                if (k <= up1) un0.y = pmin(un0.y, padd(pwt, av[k].y));
                            }
                            pwt = padd(pwt, mlbase);
                        }
                    }
                    u32 pwt = 0u;   // ta5 * MLbase
                    const int ta5 = ta < 5 ? 5 : ta;
                    for (int k = 0; k < ta5; k++) pwt = padd(pwt, mlbase);
                    for (int t0 = ta5; t0 <= tb; t0 += MFQ_MCH) {
                        uint2 av[MFQ_MCH], rv[MFQ_MCH];
#ifndef MFQ_NO_ASM
                        static_assert(MFQ_MCH == 8, "the batch below reads 8 + 8 cells");
                        {   // the chunk's 16 reads in one batch (see mfe_quad_blocks.inc)
                            const uint32_t pa = aqm1 + uint32_t(colb(j) + i - 1 + t0) * 8u;
                            const uint32_t pr = aqm + uint32_t(rowb(i, N) - 5 + t0) * 8u;
                            asm volatile(
                                "ds_read_b64 %0, %16 offset:0\n ds_read_b64 %1, %16 offset:8\n"
                                "ds_read_b64 %2, %16 offset:16\n ds_read_b64 %3, %16 offset:24\n"
                                "ds_read_b64 %4, %16 offset:32\n ds_read_b64 %5, %16 offset:40\n"
                                "ds_read_b64 %6, %16 offset:48\n ds_read_b64 %7, %16 offset:56\n"
                                "ds_read_b64 %8, %17 offset:0\n ds_read_b64 %9, %17 offset:8\n"
                                "ds_read_b64 %10, %17 offset:16\n ds_read_b64 %11, %17 offset:24\n"
                                "ds_read_b64 %12, %17 offset:32\n ds_read_b64 %13, %17 offset:40\n"
                                "ds_read_b64 %14, %17 offset:48\n ds_read_b64 %15, %17 offset:56\n"
                                "s_waitcnt lgkmcnt(0)"
                                : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]),
                                  "=&v"(av[6]), "=&v"(av[7]), "=&v"(rv[0]), "=&v"(rv[1]), "=&v"(rv[2]), "=&v"(rv[3]),
                                  "=&v"(rv[4]), "=&v"(rv[5]), "=&v"(rv[6]), "=&v"(rv[7])
                                : "v"(pa), "v"(pr)
                                : "memory");
                        }
#else
#pragma unroll
                        for (int k = 0; k < MFQ_MCH; k++) { av[k] = A1[t0 + k]; rv[k] = R[t0 + k]; }
#endif
                        u32 pw1 = padd(pwt, mlbase);
                        if (t0 + MFQ_MCH - 1 <= tb && !umask) {
#pragma unroll
                            for (int k = 0; k < MFQ_MCH; k += 2) {
                                sp0 = qmin(sp0, qadd2(rv[k], av[k]));
                                sp1 = qmin(sp1, qadd2(rv[k + 1], av[k + 1]));
                                un0 = qmin(un0, qadd(av[k], pwt));
                                un1 = qmin(un1, qadd(av[k + 1], pw1));
                                pwt = padd(pwt, mlb2);
                                pw1 = padd(pw1, mlb2);
                            }
                        } else {
#pragma unroll
                            for (int k = 0; k < MFQ_MCH; k++) {
                                const int t = t0 + k;
                                if (t <= tb) {
                                    sp0 = qmin(sp0, qadd2(rv[k], av[k]));
                                    if (t <= up0) un0.x = pmin(un0.x, padd(pwt, av[k].x));
                                    if (t <= up1) un0.y = pmin(un0.y, padd(pwt, av[k].y));
                                }
                                pwt = padd(pwt, mlbase);
                            }
                        }
                    }
                    split = qmin(sp0, sp1);
                    unp = qmin(un0, un1);
                };
                auto mstore = [&](int i, bool valid, uint2 split, uint2 unp) {
                    if (valid) {
                        L.qm[rowb(i, N) + s - 4] = qfin(qmin(split, unp));
                        L.mla[(s & 1) * NP + i] = qfin(split);
                    }
                };
                uint2 sp, un;
                int i;
                bool valid;
                if (Lm == 1 && T >= 24) {
                    const int tmid = 5 + ((((T - 4) >> 1) + 7) & ~7);
                    if (wid == WM1) {   // upper split points -> LDS, then the flag
                        mrow(0, tmid, T, sp, un, i, valid);
                        L.mpart[lane] = sp;
                        L.mpart[WAVE + lane] = un;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                        if (lane == 0) __hip_atomic_store(L.mflag, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {            // lower split points + prefix, then the combine
                        mrow(0, 0, tmid - 1, sp, un, i, valid);
                        while (__hip_atomic_load(L.mflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != d)
                            __builtin_amdgcn_s_sleep(1);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                        mstore(i, valid, qmin(sp, L.mpart[lane]), qmin(un, L.mpart[WAVE + lane]));
                    }
                } else {
                    for (int ls = (wid == WM0 ? 0 : 1); ls < Lm; ls += 2) {
                        mrow(ls, 0, T, sp, un, i, valid);
                        mstore(i, valid, sp, un);
                    }
                }
            }
        }
        QSTAMP(3);
        // ---------------- Q: q5[j], j = d - 1
        const int jq = d - 1;
        if (wid == WQ && jq >= 5 && jq <= N && (!incr || jq >= m_lo - 1)) {
            const int sj = L.S[jq];
            const int sjp = (jq < N) ? L.S[jq + 1] : 5;
            uint2 acc = qinf();
            for (int k0 = 1; k0 <= jq - 4; k0 += WAVE) {
                const int kk = k0 + lane;
                const bool ok = kk <= jq - 4;
                const int k = ok ? kk : 1;
                const int ix = off(jq - k, N) + k - 1;
                const int ty = ptype(L.S[k], sj);
                const u32 ex = L.dt[DT_EXT + ty * 36 + ((k > 1) ? L.S[k - 1] : 5) * 6 + sjp];
                const uint2 t = qadd(qadd2(L.q5[k - 1], L.qbm[ix]), padd(L.ct[CT_INVMM + L.cc[ix]], ex));
                acc = qmin(acc, ok ? t : qinf());
            }
            const u32 r0 = wave_min(acc.x), r1 = wave_min(acc.y);
            if (lane == 0) {
                const uint2 p = L.q5[jq - 1];
                L.q5[jq] = qfin(make_uint2(pmin((L.up[0][jq] >= 1) ? p.x : INF16, r0),
                                           pmin((L.up[1][jq] >= 1) ? p.y : INF16, r1)));
            }
        }
        QSTAMP(4);
        lds_barrier();
        QSTAMP(5);
    }
#ifdef ADX_STAMP
    if (lane == 0 && wid < 16)
        for (int k = 0; k < 8; k++) atomicAdd(&g_stamps_q[wid][k], st_acc[k]);
#endif
    z = L.q5[N];
    const size_t C = size_t(ka.cells);
#pragma unroll
    for (int g = 0; g < 2; g++) {
        u32 *dp = inc.dst[g];
        if (!dp) continue;
        for (int k = tid; k < int(C); k += NT) {
            dp[k] = g ? L.qbm[k].y : L.qbm[k].x;
            dp[C + k] = g ? L.qm[k].y : L.qm[k].x;
            dp[2 * C + k] = g ? L.qm1[k].y : L.qm1[k].x;
        }
        for (int k = tid; k <= N; k += NT) dp[3 * C + k] = g ? L.q5[k].y : L.q5[k].x;
    }
    // exactness guard of the 16-bit encoding: every stored value >= floor
    bool low = false;
    const int Cn = ((N - 4) * (N - 3)) >> 1;
    auto chk = [&](uint2 x) {
        const s16x2 a = sv(x.x), b = sv(x.y);
        low |= (a.x < MFE16_FLOOR) || (a.y < MFE16_FLOOR) || (b.x < MFE16_FLOOR) || (b.y < MFE16_FLOOR);
    };
    for (int k = tid; k < Cn; k += NT) {
        chk(L.qbm[k]);
        chk(L.qm[k]);
        chk(L.qm1[k]);
    }
    for (int k = tid; k <= N; k += NT) chk(L.q5[k]);
    bad = __syncthreads_or(low);
}

__device__ __noinline__ double mfq_combine(const KArgs &ka, const double *G, double *terms_out) {
    const DevScaled &X = *ka.X;
    double score = 0.0;
    for (int c = 0; c < ka.n_ctx_eff; c++) {
        for (int t = 0; t < ka.n_terms; t++) {
            const DevTermMap m = ka.tmap[c * ka.n_terms + t];
            const double gt = static_cast<double>(static_cast<float>(G[m.vfree]));
            const double ga = static_cast<double>(static_cast<float>(G[m.vcons]));
            double p = exp((gt - ga) / X.kT);
            if (!m.favorable) p = 1.0 - p;
            const double val = log(p);
            if (terms_out) terms_out[c * ka.n_terms + t] = val;
            score += m.weight * val;
        }
    }
    return score;
}

template <int NT, int NM>
__global__ void __launch_bounds__(NT, 4)
mfe_quad_kernel(KArgs ka, const DevScaled *__restrict__ XS, const DevTables *__restrict__ TT, const uint8_t *seqs,
                int W, double *scores, double *terms, float *dG, const int *mask) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const QL L = QLay<NM>::carve(smem);
    const int w = blockIdx.x;
    if (w >= W) return;
    if (ka.ovf && threadIdx.x == 0) ka.ovf[w] = 0;
    if (mask && mask[w] != 1) return;   // MC: only walkers whose proposal changed
    {
        const u32 *gct = reinterpret_cast<const u32 *>(XS->ctab);
        for (int k = threadIdx.x; k < CT_SIZE; k += NT) L.ct[k] = gct[k];
        const DevTables &T = *TT;
        const DevScaled &X = *XS;
        auto bits = [](float f) { return __float_as_uint(f); };
        for (int k = threadIdx.x; k < 200; k += NT) {
            L.dt[DT_MMH + k] = bits((&T.mmH[0][0][0])[k]);
            L.dt[DT_MMI + k] = bits((&T.mmI[0][0][0])[k]);
            L.dt[DT_MLS + k] = bits((&T.mlstem[0][0][0])[k]);
        }
        for (int k = threadIdx.x; k < 288; k += NT) L.dt[DT_EXT + k] = bits((&T.ext[0][0][0])[k]);
        for (int k = threadIdx.x; k < 8; k += NT) L.dt[DT_TAU + k] = bits(T.termAU[k]);
        for (int k = threadIdx.x; k <= ka.Nmax; k += NT) L.pw[k] = bits(X.pwml[k]);
        for (int k = threadIdx.x; k < ka.Nraw; k += NT) L.raw[k] = seqs[size_t(w) * ka.Nraw + k];
        u32 *ku = reinterpret_cast<u32 *>(L.ku);
        for (int k = threadIdx.x; k < 32 * 8; k += NT) {
            const int u = k >> 3, f = k & 7;
            const u32 *il = reinterpret_cast<const u32 *>(X.il), *nin = reinterpret_cast<const u32 *>(X.nin);
            u32 v = 0u;
            if (f < 6) v = (u >= 6 && u <= 30) ? il[u] + nin[f] : 0u;
            else if (f == 6) v = gct[CT_FB + u];
            else v = u >= 1 ? gct[CT_F1N + u - 1] : INF16;
            ku[k] = v;
        }
    }
    __syncthreads();
    bool any_bad = false;
    // pair the groups of one context (same sequence): word x = group ga, word y = group gb
    for (int ga = 0; ga < ka.n_groups2;) {
        int gb = ga;
        if (ga + 1 < ka.n_groups2) {
            const DevVariant &va = ka.variants[ka.groups2[2 * ga]], &vb = ka.variants[ka.groups2[2 * (ga + 1)]];
            if (va.ctx == vb.ctx && va.N == vb.N) gb = ga + 1;
        }
        IncQ inc{{nullptr, nullptr}, {nullptr, nullptr}, 0, 0};
        if (ka.tab) {   // MC state: read the current tables, write this proposal's
            const size_t Gf = inc_group_floats(ka.cells, ka.Nmax, 1);
            const int cur = ka.cur_slot[w];
            float *base = ka.tab + size_t(w) * 2 * ka.tab_slot;
            const bool from = ka.tab_valid[w] && ka.chg && ka.chg[2 * w] >= 0;
            const int gs[2] = {ga, gb};
            for (int h = 0; h < 2; h++) {
                const int g = gs[h];
                if (h == 1 && gb == ga) break;   // one group: word y is not kept
                inc.dst[h] = reinterpret_cast<u32 *>(base + size_t(1 - cur) * ka.tab_slot + size_t(g) * Gf);
                if (from) inc.src[h] = reinterpret_cast<const u32 *>(base + size_t(cur) * ka.tab_slot + size_t(g) * Gf);
            }
            if (from) {
                if (gb == ga) inc.src[1] = inc.src[0];
                const int lb = ka.variants[ka.groups2[2 * ga]].before_len;
                inc.m_lo = ka.chg[2 * w] + 1 + lb;
                inc.m_hi = ka.chg[2 * w + 1] + 1 + lb;
            }
        }
        uint2 z = qinf();
        bool bad = false;
        mfq_fold<NT, NM>(ka, XS, TT, ga, gb, L, z, bad, inc);
        any_bad |= bad;
        if (threadIdx.x == 0) {
            const int gs[2] = {ga, gb};
            const u32 zz[2] = {z.x, z.y};
            for (int h = 0; h < 2; h++) {
                const s16x2 q = sv(zz[h]);
                L.G[ka.groups2[2 * gs[h]]] = (q.x >= 0x4000) ? double(MFE_BIG) : static_cast<double>(q.x);
                L.G[ka.groups2[2 * gs[h] + 1]] = (q.y >= 0x4000) ? double(MFE_BIG) : static_cast<double>(q.y);
            }
        }
        __syncthreads();   // the next pair rewrites the tables
        ga = gb + 1;
    }
    if (threadIdx.x == 0) {
        for (int v = 0; v < ka.n_variants; v++) {
            const double g = (L.G[v] >= 0.5 * double(MFE_BIG)) ? double(INFINITY) : L.G[v] / 100.0;
            L.G[v] = g;
            if (dG) dG[size_t(w) * ka.n_variants + v] = static_cast<float>(g);
        }
        const int nt = ka.n_terms * ka.n_ctx_eff;
        scores[w] = mfq_combine(ka, L.G, terms ? terms + size_t(w) * nt : nullptr);
        if (any_bad && ka.ovf) {
            ka.ovf[w] = 1;                         // re-folded by the FP32 MinPlus kernel
            if (ka.tab) ka.tab_valid[w] = 0;       // and folded from scratch next time
        }
    }
}

template <int NM>
static hipError_t launch_q(const KArgs &ka, const uint8_t *seqs, int W, double *scores, double *terms, float *dG,
                           const int *mask, hipStream_t stream) {
    constexpr size_t lds = QLay<NM>::BYTES;
    static_assert(lds + 256 <= 160 * 1024, "one walker per CU (256 B static LDS)");
    auto k = mfe_quad_kernel<QWV * WAVE, NM>;
    static bool configured = false;
    if (!configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = true;
    }
    hipLaunchKernelGGL(k, dim3(W), dim3(QWV * WAVE), lds, stream, ka, ka.X, ka.T, seqs, W, scores, terms, dG, mask);
    return hipGetLastError();
}

}  // namespace

// LDS bytes of the four-fold MFE kernel for this workload (0: not covered)
size_t mfe_quad_lds(const KArgs &ka) {
    static_assert(MFQ_KSAT == 5, "host check in adx_api.cpp upload_mfe16 assumes k >= 5 saturates");
    if (!ka.mfe_cells_ok || ka.n_pairs > 0 || ka.n_variants > MFQ_MAXVAR) return 0;
    if (ka.Nmax <= 64) return QLay<64>::BYTES;
    if (ka.Nmax <= 100) return QLay<100>::BYTES;
    return 0;
}

hipError_t launch_mfe_quad(const KArgs &ka, const uint8_t *seqs, int W, double *scores, double *terms, float *dG,
                           const int *mask, hipStream_t stream) {
    if (ka.Nmax <= 64) return launch_q<64>(ka, seqs, W, scores, terms, dG, mask, stream);
    if (ka.Nmax <= 100) return launch_q<100>(ka, seqs, W, scores, terms, dG, mask, stream);
    return hipErrorInvalidValue;
}

}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_quad(unsigned long long *out, int reset) {  // [16][16]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_q), sizeof(adx::g_stamps_q)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_q), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
