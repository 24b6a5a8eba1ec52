// gfx950 minimum-free-energy fold for the Monte Carlo score (BASELINE
// configs[1]) with TWO anti-diagonals per barrier.  The recursion, the tables
// and the lanes = cells mapping are those of mfe_cells.hip (Zuker MFE of the
// ViennaRNA-2.x default model, dangles = 2, hard constraints, ligand motif;
// oracle/fold.c orc_mfe_energy; apo | holo packed as 16-bit halves); what
// changes is the step's dependency structure, so that one barrier serves two
// diagonals and a B lane-set holds the pairable cells of both:
//
// Step d (d = 6, 8, ...; one barrier at its end):
//   F  finalize e0 = d-2 and e1 = d-1, lanes = rows i, two cells per lane:
//      c = min(B's partials (loop sizes u >= 2), the stack and bulge-1 shapes
//      (inner spans e-2, e-3: final a step earlier), hairpin / motif,
//      multiloop closing mla(i+1, j-1) + closing), qbm = c + mismatchI,
//      qm1 = min(c + stem, qm1(i, j-1) + MLbase) (cell e1 takes cell e0's qm1
//      from the same lane), the unpaired part of qm
//      U(i, j) = min(qm1(i, j), U(i+1, j) + MLbase) (cell e1 takes U of row
//      i+1 from the next lane), qm = min(split, U)
//   B  interior-loop partials of diagonals d and d+1, loop sizes u >= 2
//      (inner spans <= d-3: final a step earlier), one lane-set over the
//      pairable cells of both; every block wave folds its partial into the
//      cell's slot with an LDS atomic min (apo and holo halves apart)
//   M  split parts of qm for spans d, d+1 (they read spans <= d-4)
//   Q  q5[d-3] and q5[d-2] in one pass over k
//   L  the pairable cells of diagonals d+2, d+3 and their B records
// Everything a phase reads was written one step earlier or before the loop,
// so the 97 diagonals of a 100-nt fold take 49 barriers instead of 97, and the
// step's fixed costs (records, counts, the B cell setup, the roles' round
// trips) are paid once per two diagonals.
//
// Every stored value goes through pfin() as in mfe_cells.hip.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "dev_types.hpp"
#include "fold_common.hpp"
#include "mfe_common.hpp"

namespace adx {

#ifdef ADX_STAMP
__device__ unsigned long long g_stamps_p[16][16];
#define PSTAMP(k) do { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_last; st_last = t_; __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif

namespace {

// waves per walker: 0..6 interior-loop blocks, 7 the finalize; the split parts
// of qm (one span per wave), the lists and q5 ride on block waves, whose loop
// sizes the generator partitions around them (tools/gen_mfe_blocks.py
// PAIR_ROLES4; two workgroups per CU)
#ifndef ADX_PAIR_NBLK
#define ADX_PAIR_NBLK 7
#endif
// eight waves (ten waves with nine blocks measured -37 %: a 10-wave workgroup's
// waves land 3, 3, 2, 2 on the SIMDs, so a second one does not fit at 96 VGPRs)
constexpr int NWV = 8;
constexpr int F_WAVE = 7;
#ifndef ADX_PRIO_ROLE
#define ADX_PRIO_ROLE 2
#endif
constexpr int PRIO_ROLE = ADX_PRIO_ROLE;   // s_setprio of the one-wave roles over the block waves

// (A/B round 6: a block on the finalize wave too, ADX_GEN_PAIR_NBLK=8, measured
// -5.7 %: the finalize wave then sets the step; nine block waves in ten -37 %)
#include "mfe_pair_blocks.inc"
static_assert(MFE_NBLK == ADX_PAIR_NBLK, "one block per block wave");

constexpr int PINF = 32767;   // an impossible half, sign-extended (the partial slots)

// bit 8 * log2(lanes per cell) + b: block b reads loop size u in that mode
constexpr unsigned size_bits(int u) {
    unsigned m = 0;
    for (int s = 0; s < 3; s++)
        if (MFE_SIZE_BLOCK[s][u] >= 0) m |= 1u << (8 * s + MFE_SIZE_BLOCK[s][u]);
    return m;
}

// ---------------------------------------------------------------- LDS carve
struct CP {
    u32 *qbm, *qm, *qm1;   // cell tables (fold_common.hpp indexing); qbm has an
                           // impossible "span 3" diagonal right before it
    int *part;             // [4][2][np]: B's partial minima of a diagonal (span & 3) by row,
                           //   apo / holo halves sign-extended (ds_min_i32)
    u32 *mla;              // [6][np]: split part of qm by span % 6, by row
    u32 *colmin;           // [4][np]: U(j - span, j) by span & 3, by column j
    u32 *q5;               // [np]
    u32 *ct;               // CT_SIZE (DevScaled::ctab, packed)
    u32 *dt;               // DT_* block (packed)
    uint8_t *cc;           // inner-pair code per cell (diagonal-major), pad before it
    uint8_t *S, *up, *dn, *ptn, *enc, *flg, *mat, *raw;
    u32 *pos;              // [np]: S | flg << 3 | up << 8 | ptn << 16 | enc << 24 (the per-cell pass)
    uint8_t *cl;           // [3][2 np]: rows of the pairable cells of a step's two diagonals, by step % 3
    int *cnt;              // [3]: cells of the step's first diagonal | of both << 16
    int *flag;             // [2]: block_or words (constrained, 16-bit range left)
    u32 *rec;              // [3][2][64]: the B cells' setup (rank < 64 over both diagonals) by step % 3:
                           //   i | oc << 8 | A << 16 | B << 24 and mismatchI(oc) | mismatch1n(oc) +
                           //   mismatchI(oc) << 16 (MFE table entries are equal in both halves)
    u32 *e4;               // [MFE_E4_SLOTS][4]: per-slice generic energies of the 4-lane blocks
    int np;
};

constexpr size_t al16(size_t b) { return (b + 15) & ~size_t(15); }
constexpr int MFE_E4_MAX = 64;
template <int NM>
struct PLay {
    static constexpr int NP = NM + 2;
    static constexpr size_t C = size_t(NM - 4) * (NM - 3) / 2;
    static constexpr size_t PADQ = al16(size_t(NM - 3) * 4);   // the span-3 diagonal of qbm (impossible)
    static constexpr size_t QBM = PADQ;
    static constexpr size_t QM = QBM + al16(C * 4);
    static constexpr size_t QM1 = QM + al16(C * 4);
    static constexpr size_t PART = QM1 + al16(C * 4);          // PART, MLA, CMN: the setup's scratch too
    static constexpr size_t MLA = PART + al16(4 * 2 * NP * 4);
    static constexpr size_t CMN = MLA + al16(6 * NP * 4);
    static constexpr size_t Q5 = CMN + al16(4 * NP * 4);
    static constexpr size_t CT = Q5 + al16(NP * 4);
    static constexpr size_t DT = CT + al16(CT_SIZE * 4);
    static constexpr size_t CC = DT + al16(size_t(DT_HP) * 4) + al16(NM - 3);   // span-3 codes before it
    static constexpr size_t BY = CC + al16(C);
    static constexpr size_t CLS = BY + al16(8 * NP);
    static constexpr size_t CNT = CLS + al16(6 * NP);
    static constexpr size_t FLAG = CNT + 16;
    static constexpr size_t REC = FLAG + 16;
    static constexpr size_t E4 = REC + 3 * 2 * 64 * 4;
    static constexpr size_t POS = E4 + size_t(MFE_E4_MAX) * 16;
    static constexpr size_t BYTES = POS + al16(size_t(NP) * 4);
    __device__ static CP carve() {   // LDS addresses as literals (no static LDS: the dynamic block starts at 0)
        CP l;
        l.qbm = lds_at<u32>(QBM);
        l.qm = lds_at<u32>(QM);
        l.qm1 = lds_at<u32>(QM1);
        l.part = lds_at<int>(PART);
        l.mla = lds_at<u32>(MLA);
        l.colmin = lds_at<u32>(CMN);
        l.q5 = lds_at<u32>(Q5);
        l.ct = lds_at<u32>(CT);
        l.dt = lds_at<u32>(DT);
        l.cc = lds_at<uint8_t>(CC);
        uint8_t *y = lds_at<uint8_t>(BY);
        l.S = y;
        l.up = y + NP;
        l.dn = y + 2 * NP;
        l.ptn = y + 3 * NP;
        l.enc = y + 4 * NP;
        l.flg = y + 5 * NP;
        l.mat = y + 6 * NP;
        l.raw = y + 7 * NP;
        l.cl = lds_at<uint8_t>(CLS);
        l.cnt = lds_at<int>(CNT);
        l.flag = lds_at<int>(FLAG);
        l.rec = lds_at<u32>(REC);
        l.e4 = lds_at<u32>(E4);
        l.pos = lds_at<u32>(POS);
        l.np = NP;
        return l;
    }
};
static_assert(MFE_E4_SLOTS <= MFE_E4_MAX, "CP::e4 holds the generated slots");

struct IncM {
    const u32 *src;
    u32 *dst;
    int m_lo, m_hi;
    const uint4 *cc_src;   // the slots' per-cell codes (dev_types.hpp inc_cc_offset)
    uint4 *cc_dst;
};

__device__ __forceinline__ int lanesets(int n) { return (n + 63) >> 6; }
__device__ __forceinline__ int sext_lo(u32 x) { return int(short(x & 0xFFFFu)); }
__device__ __forceinline__ int sext_hi(u32 x) { return int(x) >> 16; }
__device__ __forceinline__ u32 pack2(int lo, int hi) { return (u32(lo) & 0xFFFFu) | (u32(hi) << 16); }

// One instance per wave (WID): every wave's sweep holds only its own interior-loop
// block and roles, so the registers of the other waves' roles are not live in it
// The fold's setup (sequence, tables, refold restore, per-cell pass) and its
// write-back run in the kernel body, one copy of the code for all eight waves
// (round 6: as part of the per-wave instances each wave fetched its own copy,
// ~1.1k instruction-cache misses per fold group, profiles/r06u_icache_pmc.txt).
// Returns the constrained flag; sst (stamp builds) gets the phase cycles.
template <int NT, int NM>
__device__ __forceinline__ bool pair_setup(const KArgs &ka, const DevScaled *__restrict__ XS,
                                           const DevTables *__restrict__ TT, const int *vs, const uint8_t *raw,
                                           const CP &L, const IncM &inc, unsigned long long *sst) {
    static_assert(NT == NWV * WAVE, "one wave per block slot");
    const DevVariant V = ka.variants[vs[0]];
    const bool mh0 = ka.variants[vs[0]].motif != 0, mh1 = ka.variants[vs[1]].motif != 0;
    const int N = uni(V.N);
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);
    const int NP = L.np;
    const u32 *gct = reinterpret_cast<const u32 *>(XS->ctab);
#ifdef ADX_STAMP
    const unsigned long long st_setup0 = __builtin_amdgcn_s_memtime();
#endif
    const bool incr = inc.src != nullptr;
    const int m_lo = uni(inc.m_lo), m_hi = uni(inc.m_hi);
    // changed rows of span dd (cells containing a changed position; mfe_cells.hip)
    auto clo = [&](int dd) { return incr ? max(1, m_lo - 1 - dd) : 1; };
    auto chi = [&](int dd) { return incr ? min(N - dd, m_hi + 1) : N - dd; };
    auto qlo = [&](int s) { return incr ? max(1, m_lo - 2 - s) : 1; };
    auto qhi = [&](int s) { return incr ? min(N - s, m_hi + 2) : N - s; };

    // ---- setup loads (round 6): every table element and sequence / constraint byte this
    // thread stores, all in flight at once and stored before the restore's loads are
    // issued (the kernel prologue's loop per table waited on each load in turn, and the
    // setup tables' loads waited behind the restore's)
    static_assert(NT >= 288 && NT >= MAX_SPECIAL_HP && NT >= MAX_MOTIF && NT >= MFE_E4_SLOTS * 4 && NT >= NM + 2,
                  "one setup element per thread");
    constexpr int NCT = (CT_SIZE + NT - 1) / NT;
    u32 v_ct[NCT];
#pragma unroll
    for (int t = 0; t < NCT; t++) v_ct[t] = gct[min(tid + t * NT, CT_SIZE - 1)];
    const DevTables &T0 = *TT;
    const u32 v_mh = __float_as_uint((&T0.mmH[0][0][0])[min(tid, 199)]);
    const u32 v_mi = __float_as_uint((&T0.mmI[0][0][0])[min(tid, 199)]);
    const u32 v_ms = __float_as_uint((&T0.mlstem[0][0][0])[min(tid, 199)]);
    const u32 v_ex = __float_as_uint((&T0.ext[0][0][0])[min(tid, 287)]);
    const u32 v_tau = __float_as_uint(T0.termAU[tid & 7]);
    const u32 v_hp = __float_as_uint(XS->hp[min(tid, N)]);   // hairpin length factors (per-cell pass)
    const int ke = min(tid, MFE_E4_SLOTS * 4 - 1);
    const int e4a = MFE_E4_A[ke >> 2][ke & 3], e4u = MFE_E4_U[ke >> 2];
    const int n_sp = XS->n_special;
    const uint32_t v_spk = XS->sp_key[min(tid, MAX_SPECIAL_HP - 1)];
    const u32 v_spv = __float_as_uint(XS->sp_val[min(tid, MAX_SPECIAL_HP - 1)]);
    const uint8_t v_mc = XS->motif_code[min(tid, MAX_MOTIF - 1)];
    const int8_t v_mp = XS->motif_pt[min(tid, MAX_MOTIF - 1)];
    // position k = tid: its base (ViennaRNA's S1 wrap-around at 0 and N + 1) and constraints
    const uint8_t *cons = ka.cons + V.cons_off;
    const int np = N + 2;
    const int kp = min(tid, np - 1);
    uint8_t v_sw, v_up, v_dn, v_pt, v_en, v_fl;
    {
        const uint8_t *bef = nullptr, *aft = nullptr;
        int blen = 0;
        if (V.ctx >= 0) {
            bef = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 0];
            blen = ka.ctx_off[4 * V.ctx + 1];
            aft = ka.ctx_seq + ka.ctx_off[4 * V.ctx + 2];
        }
        const int pp = (kp == 0 ? N : (kp == N + 1 ? 1 : kp)) - 1;
        const uint8_t *sp = pp < blen ? bef + pp : (pp < blen + ka.Nraw ? raw + (pp - blen) : aft + (pp - blen - ka.Nraw));
        v_sw = *sp;
        v_up = cons[kp];
        v_dn = cons[np + kp];
        v_pt = cons[2 * np + kp];
        v_en = cons[3 * np + kp];
        v_fl = cons[4 * np + kp];
    }
    // ---- the stores: sequence, constraint arrays (mfe_cells.hip), tables
    if (tid < np) {
        L.S[tid] = v_sw;
        L.up[tid] = v_up;
        L.dn[tid] = v_dn;
        L.ptn[tid] = v_pt;
        L.enc[tid] = v_en;
        L.flg[tid] = v_fl;
        L.mat[tid] = 0;
        L.pos[tid] = u32(v_sw) | (u32(v_fl & 7) << 3) | (u32(v_up) << 8) | (u32(v_pt) << 16) | (u32(v_en) << 24);
    }
    const bool cst = tid >= 1 && tid <= N && (v_fl || v_pt);
#pragma unroll
    for (int t = 0; t < NCT; t++)
        if (tid + t * NT < CT_SIZE) L.ct[tid + t * NT] = v_ct[t];
    if (tid < 200) {
        L.dt[DT_MMH + tid] = v_mh;
        L.dt[DT_MMI + tid] = v_mi;
        L.dt[DT_MLS + tid] = v_ms;
    }
    if (tid < 288) L.dt[DT_EXT + tid] = v_ex;
    if (tid < 8) L.dt[DT_TAU + tid] = v_tau;
    u32 *hpf = L.colmin;   // the U slots' space until the sweep (initialised after the per-cell pass)
    static_assert(4 * (NM + 2) >= NM + 1, "hairpin factors fit the U slots");
    if (tid <= N) hpf[tid] = v_hp;
    // setup scratch in the partial / split / U slots (first written after the per-cell pass)
    uint32_t *spk = reinterpret_cast<uint32_t *>(L.part);
    u32 *spv = spk + MAX_SPECIAL_HP;
    uint8_t *mcode = reinterpret_cast<uint8_t *>(spk + 2 * MAX_SPECIAL_HP);
    int8_t *mpt = reinterpret_cast<int8_t *>(mcode + MAX_MOTIF);
    static_assert(2 * MAX_SPECIAL_HP * 4 + 2 * MAX_MOTIF <= PLay<NM>::MLA - PLay<NM>::PART, "setup tables fit the partials");
    if (tid < MAX_SPECIAL_HP) {
        const bool on = tid < n_sp;
        spk[tid] = on ? v_spk : 0xFFFFFFFFu;
        spv[tid] = on ? v_spv : INF16;
    }
    if (tid < MAX_MOTIF) {
        mcode[tid] = v_mc;
        mpt[tid] = v_mp;
    }
    for (int k = tid; k < NM - 3; k += NT) {   // the impossible span-3 diagonal (B's d-lanes reach it)
        (L.qbm - (NM - 3))[k] = INF16;
        (L.cc - (NM - 3))[k] = 0;
    }

    // ---- refold restore: the loads of all three tables (8-byte vector loads into
    // registers), stored to LDS after the motif scan, so their HBM latency overlaps
    // it (round 6; the loop of dependent load -> store pairs cost ~20k cycles per
    // fold group).  The generic interior energies of the 4-lane blocks (e4) ride along.
    const u32 v_e4 = XS->ku16[e4u][max(e4a, 0)];
    constexpr int CNM = ((NM - 4) * (NM - 3)) >> 1;
    constexpr int RS = (3 * (CNM >> 1) + NT - 1) / NT;   // loads per thread
    const int Crs = ((N - 4) * (N - 3)) >> 1, half = Crs >> 1;
    uint2 rsv[RS];
    constexpr int RC = (((CNM + 15) >> 4) + NT - 1) / NT;   // per-cell code loads per thread (uint4)
    const int C16 = (Crs + 15) >> 4;
    uint4 rcv[RC];
    u32 rod = 0, r5 = 0;   // the odd last cell of each table, q5's prefix
    if (incr) {
        const size_t Cs = size_t(ka.cells);
#pragma unroll
        for (int t = 0; t < RS; t++) {
            const int k = tid + t * NT;
            const int kk = k < 3 * half ? k : 0;
            const int a = kk / half, c = kk - a * half;
            rsv[t] = *reinterpret_cast<const uint2 *>(inc.src + a * Cs + 2 * c);
        }
#pragma unroll
        for (int t = 0; t < RC; t++) {
            const int k = tid + t * NT;
            rcv[t] = inc.cc_src[k < C16 ? k : 0];
        }
        rod = inc.src[min(tid, 2) * Cs + max(Crs - 1, 0)];
        r5 = inc.src[3 * Cs + min(tid, N)];
    } else {
        const int C = ((N - 4) * (N - 3)) >> 1;
        for (int k = tid; k < C; k += NT) L.qm[k] = INF16;
    }
#ifdef ADX_STAMP
    const unsigned long long st_s1 = __builtin_amdgcn_s_memtime();   // setup tables stored, restore issued
#endif
    const bool constrained = block_or(L.flag, cst);
    const int mL = XS->motif_len;
#ifdef ADX_STAMP
    const unsigned long long st_s2 = __builtin_amdgcn_s_memtime();   // sequence, constraints
#endif
    if ((mh0 || mh1) && mL > 0) {
        // lanes = starts; the motif's positions in chunks of 8 independent reads (one
        // LDS round trip per chunk, not one per position of the longest match)
        for (int o0 = 1 + wid * WAVE; o0 + mL - 1 <= N; o0 += NT) {
            const int o = o0 + lane;
            const bool in = o + mL - 1 <= N;
            bool ok = in;
            for (int k0 = 0; k0 < mL; k0 += 8) {
                uint32_t sb[8], mb[8];
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    sb[t] = L.S[min(o + k0 + t, N + 1)];
                    mb[t] = mcode[k0 + t];
                }
#pragma unroll
                for (int t = 0; t < 8; t++) ok = ok && (k0 + t >= mL || sb[t] == mb[t]);
                if (__ballot(ok) == 0) break;
            }
            if (in) L.mat[o] = ok ? 1 : 0;
        }
        __syncthreads();
        for (int o = 1 + wid; o + mL - 1 <= N; o += NT / WAVE) {
            if (!uni(L.mat[o])) continue;
            bool ok = true;
            for (int k = lane; k < mL; k += WAVE) {
                const int pk = mpt[k];
                if (pk < 0) ok = ok && L.up[o + k] >= 1;
                else if (pk > k) ok = ok && allowed(L, o + k, o + pk);
            }
            const bool all = __ballot(!ok) == 0;
            if (lane == 0) L.mat[o] = all ? 1 : 0;
        }
    }
#ifdef ADX_STAMP
    const unsigned long long st_s25 = __builtin_amdgcn_s_memtime();   // motif scan done
#endif
    if (incr) {   // the restore's stores (loads issued at the start)
        const size_t Cs = size_t(ka.cells);
#pragma unroll
        for (int t = 0; t < RS; t++) {
            const int k = tid + t * NT;
            if (k < 3 * half) {
                const int a = k / half, c = k - a * half;
                u32 *d = a == 0 ? L.qbm : a == 1 ? L.qm : L.qm1;
                *reinterpret_cast<uint2 *>(d + 2 * c) = rsv[t];
            }
        }
        if ((Crs & 1) && tid < 3) (tid == 0 ? L.qbm : tid == 1 ? L.qm : L.qm1)[Crs - 1] = rod;
#pragma unroll
        for (int t = 0; t < RC; t++) {   // the codes (16 cells per store; the band's are recomputed)
            const int k = tid + t * NT;
            if (k < C16) reinterpret_cast<uint4 *>(L.cc)[k] = rcv[t];
        }
        if (tid <= m_lo - 2 && tid <= N) L.q5[tid] = r5;
    }
    if (tid < MFE_E4_SLOTS * 4) L.e4[tid] = e4a < 0 ? INF16 : v_e4;
    // the per-cell pass's quarter-sets (below): diagonal d's band rows in sets of 16,
    // listed diagonal by diagonal in the split slots' space (free until the sweep)
    // by the waves of lane-sets 0, 1 of the diagonals: qtab[k] = d | first row << 8
    static_assert(NM - 4 <= 2 * WAVE, "the diagonals' quarter-set counts in two lane-sets");
    static_assert((NM - 4) + ((NM - 4) * (NM - 3) / 2 + 15) / 16 <= 6 * (NM + 2), "quarter-sets fit the split slots");
    u32 *qtab = L.mla;
    int tot = 0;  // quarter-sets
#pragma unroll
    for (int xs = 0; xs < 2; xs++) {
        const int d = 4 + xs * WAVE + lane;
        const int n = d <= N - 1 ? max(0, chi(d) - clo(d) + 1) : 0;
        const int q = (n + 15) >> 4;
        int v = q;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int t = __shfl_up(v, o, WAVE);
            if (lane >= o) v += t;
        }
        if (wid == xs)
            for (int c = 0; c < q; c++) qtab[tot + v - q + c] = u32(d) | (u32(clo(d) + 16 * c) << 8);
        tot += __shfl(v, WAVE - 1, WAVE);
    }
    tot = uni(tot);
    __syncthreads();
    const u32 mx = __float_as_uint(XS->motif_extra);
    const u32 mextra = (mh0 ? (mx & 0xFFFFu) : 0x7FFFu) | (mh1 ? (mx & 0xFFFF0000u) : 0x7FFF0000u);
    if (tid == 0) {
        L.q5[0] = 0u;
        for (int j = 1; j <= 4 && j <= N; j++) L.q5[j] = (L.up[j] >= 1) ? L.q5[j - 1] : INF16;
    }
#ifdef ADX_STAMP
    const unsigned long long st_s3 = __builtin_amdgcn_s_memtime();   // motif sites
#endif
    // ---- per-cell setup (mfe_cells.hip): inner-pair code, hairpin (+ motif) or the
    // non-pairable mark, multiloop stem of the pairable cells, for the changed band
    // (a fold from scratch: every cell; a refold restored the others).  Round 6:
    // the band's rows in quarter-sets of 16 (diagonal d, rows clo(d) + 16c ..), four
    // quarter-sets per 64-lane item and four items per batch, each batch in two LDS
    // round trips; items by diagonal left most lanes idle (a refold's band holds
    // d + 3 rows of diagonal d) and took three times the batches
    auto cell_pass = [&](int I0) __attribute__((always_inline)) {
        constexpr int NI = 4;   // items I0 .. I0 + 3 (quarter-sets 4 I .. 4 I + 3, lanes 16 g ..)
        int ii[NI], jj[NI], dv[NI];
        bool ok[NI];
        u32 wim[NI], wi[NI], wi1[NI], wjm[NI], wj[NI], wjp[NI];
        uint32_t mt[NI];
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const int k = 4 * (I0 + q) + (lane >> 4);   // the lane's quarter-set
            const u32 e = qtab[k < tot ? k : 0];
            const int d = k < tot ? int(e & 255) : 4;
            const int r = int(e >> 8) + (lane & 15) - 1;
            const bool v = k < tot && r < chi(d);
            dv[q] = d;
            ok[q] = v;
            const int i = ok[q] ? r + 1 : 1, j = ok[q] ? i + d : 5;
            ii[q] = i;
            jj[q] = j;
            wim[q] = L.pos[i - 1];
            wi[q] = L.pos[i];
            wi1[q] = L.pos[i + 1];
            wjm[q] = L.pos[j - 1];
            wj[q] = L.pos[j];
            wjp[q] = L.pos[j + 1];
            mt[q] = L.mat[i];
        }
        int ty[NI], ix1[NI];
        bool pr[NI], inb[NI];
        u32 f1[NI], f2[NI], hv[NI];
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const int i = ii[q], j = jj[q], d = dv[q];
            hv[q] = hpf[d - 1];
            const int si = wi[q] & 7, sj = wj[q] & 7;
            ty[q] = ptype(si, sj);
            inb[q] = ok[q];
            const int fi = (wi[q] >> 3) & 7, fj = (wj[q] >> 3) & 7;
            const int pi = (wi[q] >> 16) & 255, pj = (wj[q] >> 16) & 255;
            bool al = !((fi | fj) & 1) && !((fi & 2) || (fj & 4));
            al = al && (pi ? pi == j : (pj ? pj == i : (wi[q] >> 24) == (wj[q] >> 24)));
            pr[q] = inb[q] && ty[q] != 0 && al;
            const int sim = wim[q] & 7, sjp = wjp[q] & 7, si1 = wi1[q] & 7, sjm = wjm[q] & 7;
            ix1[q] = (d - 1 == 3) ? DT_TAU + ty[q] : DT_MMH + ty[q] * 25 + si1 * 5 + sjm;
            f1[q] = L.dt[ix1[q]];
            f2[q] = L.dt[DT_MLS + ty[q] * 25 + sim * 5 + sjp];
        }
#pragma unroll
        for (int q = 0; q < NI; q++) {
            const int i = ii[q], j = jj[q], d = dv[q], u = d - 1;
            if (!ok[q]) continue;
            L.cc[off(d, N) + i - 1] = static_cast<uint8_t>(rtype(ty[q]) * 25 + (wjp[q] & 7) * 5 + (wim[q] & 7));
            u32 h = INF16;
            if (((wi1[q] >> 8) & 255) >= uint32_t(u)) {
                h = padd(hv[q], f1[q]);
                if (u == 3 || u == 4 || u == 6) {   // special hairpins (three diagonals)
                    const int sh = special_hp(spk, hp_key(L.S, i, u + 2));
                    if (sh >= 0) h = spv[sh];
                }
            }
            if (d == mL - 1 && mL > 0 && mt[q]) h = pmin(h, mextra);
            if (inb[q]) {
                L.qbm[off(d, N) + i - 1] = pr[q] ? h : MARK16;
                L.qm1[colb(j) + i - 1] = pr[q] ? f2[q] : INF16;
            }
        }
    };
    for (int I0 = wid * 4; 4 * I0 < tot; I0 += NWV * 4) cell_pass(I0);
#ifdef ADX_STAMP
    const unsigned long long st_s35 = __builtin_amdgcn_s_memtime();   // this wave's cells (before the barrier)
#endif
    __syncthreads();
#ifdef ADX_STAMP
    const unsigned long long st_s4 = __builtin_amdgcn_s_memtime();   // per-cell pass
#endif
    // the partial, split and U slots start impossible (the setup used their space)
    for (int k = tid; k < 4 * 2 * NP; k += NT) L.part[k] = PINF;
    for (int k = tid; k < 6 * NP; k += NT) L.mla[k] = INF16;
    for (int k = tid; k < 4 * NP; k += NT) L.colmin[k] = INF16;
    __syncthreads();
#ifdef ADX_STAMP
    {
        const unsigned long long st_end = __builtin_amdgcn_s_memtime();
        sst[0] = st_end - st_setup0;
        sst[1] = st_s1 - st_setup0;
        sst[2] = st_s2 - st_s1;
        sst[3] = st_s25 - st_s2;
        sst[4] = st_s3 - st_s25;
        sst[5] = st_s4 - st_s3;
        sst[6] = st_s35 - st_s3;
    }
#endif
    return constrained;
}

template <int NT, int NM, int WID>
__device__ __forceinline__ void mfe_pair_fold(const KArgs &ka, const DevScaled *__restrict__ XS,
                                              const DevTables *__restrict__ TT, const int *vs, const CP &L,
                                              const IncM &inc, const bool constrained, const unsigned long long *sst) {
    const DevVariant V = ka.variants[vs[0]];
    const int N = uni(V.N);
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    constexpr int wid = WID;
    const int NP = L.np;
    const u32 *gct = reinterpret_cast<const u32 *>(XS->ctab);
    const bool incr = inc.src != nullptr;
    const int m_lo = uni(inc.m_lo), m_hi = uni(inc.m_hi);
    auto clo = [&](int dd) { return incr ? max(1, m_lo - 1 - dd) : 1; };
    auto chi = [&](int dd) { return incr ? min(N - dd, m_hi + 1) : N - dd; };
    auto qlo = [&](int s) { return incr ? max(1, m_lo - 2 - s) : 1; };
    auto qhi = [&](int s) { return incr ? min(N - s, m_hi + 2) : N - s; };
    const u32 mlclosing = __float_as_uint(XS->mlclosing);
    const u32 mlbase = __float_as_uint(XS->mlbase_sig);
    const DevTables &T = *TT;
    const u32 *T11 = reinterpret_cast<const u32 *>(&T.int11[0][0][0][0]);
    const u32 *T21 = reinterpret_cast<const u32 *>(&T.int21[0][0][0][0][0]);
    const u32 *T22 = reinterpret_cast<const u32 *>(&T.int22[0][0][0][0][0][0]);
    const u32 tauE = gct[CT_FSM + 6];
    const u32 fsm5 = gct[CT_FSM + 5];
    const u32 fs1 = gct[CT_FSM + 1];
    BUni U;
    U.qbm = L.qbm;
    U.cc = L.cc;
    U.ct = L.ct;
    U.gct = gct;
    U.kg = reinterpret_cast<const uint4 *>(XS->ku16);
    U.aq = lds_addr(L.qbm);
    U.ac = lds_addr(L.cc);
    U.act = lds_addr(L.ct);
    U.fs1 = fs1;
    U.il = reinterpret_cast<const u32 *>(XS->il);
    U.nin = reinterpret_cast<const u32 *>(XS->nin);
    U.N = N;
    const uint32_t aqm = lds_addr(L.qm), aqm1 = lds_addr(L.qm1), ae4 = lds_addr(L.e4);
    constexpr int L_WAVE = 1;           // (round 5: wave 1 +0.8 % over wave 4, A/B r05zn/r05zo) the lists two steps ahead (diagonals d+4, d+5) and their B records
    constexpr int Q_WAVE = 3;           // q5 of two columns (on the finalize wave: -2.1 %, A/B r06n)
    constexpr int fw[2] = {F_WAVE, 6};  // finalize lane-sets 0, 1 (rows 1..64, 64..127): lane-set 1
                                        // (spans < 38) rides on block wave 6
    constexpr int mw[2] = {0, 2};       // the split parts of spans d, d+1
    constexpr int fls = fw[0] == wid ? 0 : (fw[1] == wid ? 1 : -1);
    const int NP2 = 2 * NP;
    // the pairable cells of diagonals db, db+1 (ranks < P0 on db) and the B records of
    // ranks < 64 into list slot sl (a step's B reads them two steps later: its first
    // lane-set's records are loaded a step ahead, across the barrier)
    auto build_list = [&](int db, int sl) {
        int base = 0, P0 = 0;
        for (int k = 0; k < 2; k++) {
            const int dn = db + k;
            if (k == 1) P0 = base;
            if (dn < 8 || dn > N - 1) continue;   // interior loops u >= 2 need spans >= 8
            const int lo = clo(dn), hi = chi(dn);
            const int Ln = lanesets(hi - lo + 1);
            for (int ls = 0; ls < Ln; ls++) {
                const int i = lo + ls * WAVE + lane;
                const bool pr = i <= hi && L.qbm[off(dn, N) + i - 1] != MARK16;
                const uint64_t m = __ballot(pr);
                const int rk = base + __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
                if (pr) L.cl[sl * NP2 + rk] = uint8_t(i);
                if (pr && rk < WAVE) {
                    const int j = i + dn;
                    const int oc = ptype(L.S[i], L.S[j]) * 25 + L.S[i + 1] * 5 + L.S[j - 1];
                    const u32 mmo = L.dt[DT_MMI + oc];
                    u32 *rr = L.rec + sl * 2 * WAVE + rk;
                    rr[0] = uint32_t(i) | (uint32_t(oc) << 8) | (uint32_t(L.up[i + 1]) << 16) |
                            (uint32_t(L.dn[j - 1]) << 24);
                    rr[WAVE] = (mmo & 0xFFFFu) | (padd(L.ct[CT_ONEN + oc], mmo) << 16);
                }
                base += __popcll(m);
            }
        }
        if (lane == 0) L.cnt[sl] = P0 | (base << 16);
    };
    if (wid == L_WAVE) {   // steps 0 (no B work: d + 1 < 8) and 1
        if (lane == 0) L.cnt[0] = 0;
        build_list(8, 1);
    }
    __syncthreads();
    // the first lane-set's B record of the next step, loaded a step ahead
    auto slices = [](int P) { return P <= 16 ? 2 : (P <= 32 ? 1 : 0); };   // log2 slices per cell
    int cPP = 0;                // this step's list counts (CP::cnt), loaded a step ahead,
    u32 cwd = 0, cmm = 0;       // and its first lane-set's B record
    // loaded at the top of the step before (issued with nothing to wait on: they
    // complete under the step's first read batch); the records of the 4-lanes-
    // per-cell mapping (lane & 15), the one of ~96 % of a refold's steps -- B
    // reads its records itself when the step maps its lanes otherwise
    auto load_list = [&](int sl, int &PP, u32 &wd, u32 &mm) {
        PP = L.cnt[sl];
        const u32 *rr = L.rec + sl * 2 * WAVE + (lane & 15);
        wd = rr[0];
        mm = rr[WAVE];
    };
    // the record's two energies, each 16 bits wide, to packed apo | holo words
    auto lo2 = [](u32 x) { return __builtin_amdgcn_perm(x, x, 0x05040504u); };
    auto hi2 = [](u32 x) { return __builtin_amdgcn_perm(x, x, 0x07060706u); };

#ifdef ADX_STAMP
    unsigned long long st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long st_sw0 = __builtin_amdgcn_s_memtime();
    unsigned long long st_last = st_sw0;
#ifndef ADX_STAMP_F
    st_acc[11] = sst[1];
    st_acc[12] = sst[2];
    st_acc[13] = sst[3];
#endif
    st_acc[7] = sst[4];
    st_acc[14] = sst[5];
    st_acc[15] = sst[6];
#endif
#ifdef ADX_STAMP
    st_acc[8] = sst[0] + (st_last - st_sw0);   // setup + the sweep's prelude
#endif
    int sl = 0;   // list slot of this step: step index % 3
    for (int d = 6; d - 3 <= N; d += 2) {
        const int sl1 = sl == 2 ? 0 : sl + 1, sl2 = sl1 == 2 ? 0 : sl1 + 1;
        PSTAMP(0);
        int nPP = 0;
        u32 nwd = 0, nmm = 0;
        if (wid < MFE_NBLK) load_list(sl1, nPP, nwd, nmm);   // the next step's, built a step ago
        // ---------------- L: the pairable cells of diagonals d+4, d+5 (B's lanes two
        // steps on; their qbm marks are the setup's) and the records of ranks < 64
        if (wid == L_WAVE) {
            __builtin_amdgcn_s_setprio(PRIO_ROLE);
            build_list(d + 4, sl2);
            __builtin_amdgcn_s_setprio(0);
        }
        PSTAMP(1);
        // ---------------- F: finalize e0 = d-2 and e1 = d-1.  Lanes = rows i (all
        // rows: the unpaired part U is kept for every cell); a lane-set spans 64 rows,
        // consecutive lane-sets overlap by one row (lane 63 recomputes the next set's
        // first row for its U and writes nothing), so no value crosses waves.
        {
            const int e0 = d - 2, e1 = d - 1;
            const int R = N - e0;                                   // rows of span e0 (e1: R - 1)
            const int Lf = R <= 64 ? 1 : (R - 1 + 62) / 63;
            if (e0 <= N - 1 && fls >= 0 && fls < Lf) {
                __builtin_amdgcn_s_setprio(PRIO_ROLE);
                const int i0 = 1 + fls * 63 + lane;
                const bool own = lane < 63 || fls == Lf - 1;         // the overlap lane writes nothing
                const bool rowA = i0 <= R, rowB = i0 <= R - 1;
                const int i = rowA ? i0 : R;                         // every lane reads (batch)
                const int jA = i + e0;
                const int ceA = off(e0, N) + i - 1, ceB = off(e1, N) + i - 1;
                const int cmA = colb(jA) + i - 1, cmB = colb(jA + 1) + i - 1;
                // inner cells of the stack / bulge-1 shapes: spans e0-3, e0-2, e0-1
                const int s3 = max(e0 - 3, 3), s2 = max(e0 - 2, 3), s1 = max(e0 - 1, 3);
                const int c3 = off(s3, N) + i, c2 = off(s2, N) + i, c1 = off(s1, N) + i;
                u32 initA, cceA, stA, pqA, mlA, spA, upA, a0, a1, vS3, cS3, vS3b, cS3b, vS2, cS2, vS2b, cS2b, vS1, cS1;
                u32 initB, cceB, stB, mlB, spB, b0, b1;
                uint32_t si, si1, sjm, sj, sjp, ui, ui1, ujA, ujB, djm, dj;
                {
                    const uint32_t aq = U.aq, ac = U.ac;
                    const uint32_t pA = lds_addr(L.part) + uint32_t(((e0 & 3) * 2 * NP) + i) * 4u;
                    const uint32_t pB = lds_addr(L.part) + uint32_t(((e1 & 3) * 2 * NP) + i) * 4u;
                    const uint32_t mA = lds_addr(L.mla) + uint32_t(((e0 + 4) % 6) * NP + i + 1) * 4u;   // span e0-2
                    const uint32_t mB = lds_addr(L.mla) + uint32_t(((e1 + 4) % 6) * NP + i + 1) * 4u;
                    const uint32_t sA = lds_addr(L.mla) + uint32_t((e0 % 6) * NP + i) * 4u;
                    const uint32_t sB = lds_addr(L.mla) + uint32_t((e1 % 6) * NP + i) * 4u;
                    const uint32_t uA = lds_addr(L.colmin) + uint32_t(((e0 + 3) & 3) * NP + jA) * 4u;  // span e0-1
                    const uint32_t aS = lds_addr(L.S), aU = lds_addr(L.up), aD = lds_addr(L.dn);
                    asm volatile(
                        "ds_read_b32 %[initA], %[qA]\n"
                        "ds_read_u8 %[cceA], %[kA]\n"
                        "ds_read_b32 %[stA], %[q1A]\n"
                        "ds_read_b32 %[pqA], %[q1P]\n"
                        "ds_read_b32 %[mlA], %[mA]\n"
                        "ds_read_b32 %[spA], %[sA]\n"
                        "ds_read_b32 %[upA], %[uA]\n"
                        "ds_read_b32 %[a0], %[pA]\n"
                        "ds_read_b32 %[a1], %[pA] offset:%[pst]\n"
                        "ds_read_b32 %[initB], %[qB]\n"
                        "ds_read_u8 %[cceB], %[kB]\n"
                        "ds_read_b32 %[stB], %[q1B]\n"
                        "ds_read_b32 %[mlB], %[mB]\n"
                        "ds_read_b32 %[spB], %[sB]\n"
                        "ds_read_b32 %[b0], %[pB]\n"
                        "ds_read_b32 %[b1], %[pB] offset:%[pst]\n"
                        "ds_read_b32 %[vS3], %[q3]\n"
                        "ds_read_b32 %[vS3b], %[q3] offset:4\n"
                        "ds_read_b32 %[vS2], %[q2]\n"
                        "ds_read_b32 %[vS2b], %[q2] offset:4\n"
                        "ds_read_b32 %[vS1], %[q1]\n"
                        "ds_read_u8 %[cS3], %[k3]\n"
                        "ds_read_u8 %[cS3b], %[k3] offset:1\n"
                        "ds_read_u8 %[cS2], %[k2]\n"
                        "ds_read_u8 %[cS2b], %[k2] offset:1\n"
                        "ds_read_u8 %[cS1], %[k1]\n"
                        "ds_read_u8 %[si], %[aSi]\n"
                        "ds_read_u8 %[si1], %[aSi] offset:1\n"
                        "ds_read_u8 %[sjm], %[aSj] offset:0\n"
                        "ds_read_u8 %[sj], %[aSj] offset:1\n"
                        "ds_read_u8 %[sjp], %[aSj] offset:2\n"
                        "ds_read_u8 %[ui], %[aUi]\n"
                        "ds_read_u8 %[ui1], %[aUi] offset:1\n"
                        "ds_read_u8 %[ujA], %[aUj]\n"
                        "ds_read_u8 %[ujB], %[aUj] offset:1\n"
                        "ds_read_u8 %[djm], %[aDj] offset:0\n"
                        "ds_read_u8 %[dj], %[aDj] offset:1\n"
                        "s_waitcnt lgkmcnt(0)"
                        : [initA] "=&v"(initA), [cceA] "=&v"(cceA), [stA] "=&v"(stA), [pqA] "=&v"(pqA), [mlA] "=&v"(mlA),
                          [spA] "=&v"(spA), [upA] "=&v"(upA), [a0] "=&v"(a0), [a1] "=&v"(a1), [initB] "=&v"(initB),
                          [cceB] "=&v"(cceB), [stB] "=&v"(stB), [mlB] "=&v"(mlB), [spB] "=&v"(spB), [b0] "=&v"(b0),
                          [b1] "=&v"(b1), [vS3] "=&v"(vS3), [vS3b] "=&v"(vS3b), [vS2] "=&v"(vS2), [vS2b] "=&v"(vS2b),
                          [vS1] "=&v"(vS1), [cS3] "=&v"(cS3), [cS3b] "=&v"(cS3b), [cS2] "=&v"(cS2), [cS2b] "=&v"(cS2b),
                          [cS1] "=&v"(cS1), [si] "=&v"(si), [si1] "=&v"(si1), [sjm] "=&v"(sjm), [sj] "=&v"(sj),
                          [sjp] "=&v"(sjp), [ui] "=&v"(ui), [ui1] "=&v"(ui1), [ujA] "=&v"(ujA), [ujB] "=&v"(ujB),
                          [djm] "=&v"(djm), [dj] "=&v"(dj)
                        : [qA] "v"(aq + uint32_t(ceA) * 4u), [kA] "v"(ac + uint32_t(ceA)),
                          [q1A] "v"(aqm1 + uint32_t(cmA) * 4u), [q1P] "v"(aqm1 + uint32_t(colb(jA - 1) + i - 1) * 4u),
                          [mA] "v"(mA), [sA] "v"(sA), [uA] "v"(uA), [pA] "v"(pA), [pst] "i"(NM * 4 + 8),
                          [qB] "v"(aq + uint32_t(ceB) * 4u), [kB] "v"(ac + uint32_t(ceB)),
                          [q1B] "v"(aqm1 + uint32_t(cmB) * 4u), [mB] "v"(mB), [sB] "v"(sB), [pB] "v"(pB),
                          [q3] "v"(aq + uint32_t(c3) * 4u), [q2] "v"(aq + uint32_t(c2) * 4u), [q1] "v"(aq + uint32_t(c1) * 4u),
                          [k3] "v"(ac + uint32_t(c3)), [k2] "v"(ac + uint32_t(c2)), [k1] "v"(ac + uint32_t(c1)),
                          [aSi] "v"(aS + uint32_t(i)), [aSj] "v"(aS + uint32_t(jA - 1)), [aUi] "v"(aU + uint32_t(i)),
                          [aUj] "v"(aU + uint32_t(jA)), [aDj] "v"(aD + uint32_t(jA - 1))
                        : "memory");
                }
#ifdef ADX_STAMP_F
                PSTAMP(11);   // F: the read batch
#endif
                static_assert(NM + 2 == PLay<NM>::NP, "partial halves are NP words apart");
                // the loop-correction factors of the stack / bulge-1 shapes and the cells' own terms
                const int tyA = ptype(si, sj), tyB = ptype(si, sjp);
                const int t8A = tyA * 8, t8B = tyB * 8;
                auto stk = [&](u32 v, u32 c, int t8) {   // inner pair with code c closing a stack with type t8/8
                    return padd(v, padd(L.ct[CT_INVMM + c], L.ct[CT_STK + t8 + ((int(c) * 41) >> 10)]));
                };
                // A = (i, jA): stack inner (i+1, jA-1) span e0-2 [vS2]; bulges (0,1) inner
                // (i+1, jA-2) [vS3], (1,0) inner (i+2, jA-1) [vS3b], span e0-3.
                // B = (i, jA+1): stack inner (i+1, jA) span e0-1 [vS1]; bulges (0,1) inner
                // (i+1, jA-1) [vS2], (1,0) inner (i+2, jA) [vS2b], span e0-2.
                u32 iA = INF16, iB = INF16;
                if (e0 >= 6) iA = stk(vS2, cS2, t8A);
                if (e0 >= 7) {
                    iA = pmin(iA, djm >= 1 ? padd(stk(vS3, cS3, t8A), fs1) : INF16);
                    iA = pmin(iA, ui1 >= 1 ? padd(stk(vS3b, cS3b, t8A), fs1) : INF16);
                }
                if (e1 >= 6) iB = stk(vS1, cS1, t8B);
                if (e1 >= 7) {
                    iB = pmin(iB, dj >= 1 ? padd(stk(vS2, cS2, t8B), fs1) : INF16);
                    iB = pmin(iB, ui1 >= 1 ? padd(stk(vS2b, cS2b, t8B), fs1) : INF16);
                }
                const u32 mlclA = padd(mlclosing, L.dt[DT_MLS + rtype(tyA) * 25 + sjm * 5 + si1]);
                const u32 mlclB = padd(mlclosing, L.dt[DT_MLS + rtype(tyB) * 25 + sj * 5 + si1]);
                const u32 mmiA = L.dt[DT_MMI + cceA], mmiB = L.dt[DT_MMI + cceB];
                const bool inA = rowA && (!incr || (i >= clo(e0) && i <= chi(e0)));
                const bool inB = rowB && e1 <= N - 1 && (!incr || (i >= clo(e1) && i <= chi(e1)));
                // cell A
                u32 q1A = stA;   // restored qm1 outside the band
                if (inA) {
                    const u32 prev = (e0 >= 5 && ujA >= 1) ? padd(pqA, mlbase) : INF16;
                    u32 f1 = prev;
                    if (initA != MARK16) {
                        u32 c = pmin(initA, pack2(int(a0), int(a1)));
                        c = pmin(c, iA);
                        c = pfin(pmin(c, padd(mlA, mlclA)));
                        if (own) L.qbm[ceA] = pfin(padd(c, mmiA));
                        f1 = pmin(padd(c, stA), prev);
                    }
                    q1A = pfin(f1);
                    if (own) L.qm1[cmA] = q1A;
                }
                const u32 UA = ui >= 1 ? pmin(q1A, padd(upA, mlbase)) : q1A;
                // cell B (its qm1 predecessor (i, jA) is cell A of this lane)
                u32 q1B = stB;
                if (inB) {
                    const u32 prev = (e1 >= 5 && ujB >= 1) ? padd(q1A, mlbase) : INF16;
                    u32 f1 = prev;
                    if (initB != MARK16) {
                        u32 c = pmin(initB, pack2(int(b0), int(b1)));
                        c = pmin(c, iB);
                        c = pfin(pmin(c, padd(mlB, mlclB)));
                        if (own) L.qbm[ceB] = pfin(padd(c, mmiB));
                        f1 = pmin(padd(c, stB), prev);
                    }
                    q1B = pfin(f1);
                    if (own) L.qm1[cmB] = q1B;
                }
#ifdef ADX_STAMP_F
                PSTAMP(12);   // F: the cells' terms
#endif
                // U of row i+1 in column jA+1 (span e0) is the next lane's cell A
                const u32 UA1 = u32(__builtin_amdgcn_ds_bpermute((lane + 1) * 4, int(UA)));
                const u32 UB = ui >= 1 ? pmin(q1B, padd(UA1, mlbase)) : q1B;
                if (own && rowA) {
                    L.colmin[(e0 & 3) * NP + jA] = UA;
                    L.part[(e0 & 3) * 2 * NP + i] = PINF;
                    L.part[(e0 & 3) * 2 * NP + NP + i] = PINF;
                    if (e0 <= N - 3 && (!incr || (i >= qlo(e0) && i <= qhi(e0))))
                        L.qm[rowb(i, N) + e0 - 4] = pfin(pmin(e0 >= 9 ? spA : INF16, UA));
                }
                if (own && rowB && e1 <= N - 1) {
                    L.colmin[(e1 & 3) * NP + jA + 1] = UB;
                    L.part[(e1 & 3) * 2 * NP + i] = PINF;
                    L.part[(e1 & 3) * 2 * NP + NP + i] = PINF;
                    if (e1 <= N - 3 && (!incr || (i >= qlo(e1) && i <= qhi(e1))))
                        L.qm[rowb(i, N) + e1 - 4] = pfin(pmin(e1 >= 9 ? spB : INF16, UB));
                }
                __builtin_amdgcn_s_setprio(0);
#ifdef ADX_STAMP_F
                PSTAMP(13);   // F: U, the stores
#endif
            }
        }
        PSTAMP(2);
        // ---------------- B: interior-loop partials (u >= 2) of diagonals d and d+1.
        // Lanes = the pairable cells of both (listed last step: ranks < P0 on d,
        // the rest on d+1); a lane of d+1 reads its inner cells at
        // off(d - 2 - u) + i + (N - d + 2 + u), which the blocks add per lane (hb).
        if (d + 1 >= 8 && d <= N - 1) {
            const int P0 = uni(cPP & 0xFFFF), P = uni(cPP >> 16);
            const int sh = slices(P);
            const int cwl = 6 - sh;
            const int Lb = (P + (1 << cwl) - 1) >> cwl;
            constexpr int blk = wid;
            const int r = lane >> cwl;
            U.d = d;
            U.umax = d - 5 < 30 ? d - 5 : 30;   // d+1's loop sizes; d's last one reads the impossible span 3
            for (int ls = 0; ls < Lb && blk < MFE_NBLK; ls++) {
                const int idx = (ls << cwl) + (lane & ((1 << cwl) - 1));
                if (idx < P) {
                    const int hb = idx >= P0 ? 1 : 0;
                    const int dd = d + hb;
                    int i, oc, cA, cB;
                    u32 mmo, mo;
                    if (ls == 0 && sh == 2) {   // loaded a step ahead
                        const u32 wd = cwd;
                        mmo = lo2(cmm);
                        mo = hi2(cmm);
                        i = wd & 255;
                        oc = (wd >> 8) & 255;
                        cA = (wd >> 16) & 255;
                        cB = wd >> 24;
                    } else if (idx < WAVE) {
                        const u32 *rr = L.rec + sl * 2 * WAVE + idx;
                        const u32 wd = rr[0];
                        mmo = lo2(rr[WAVE]);
                        mo = hi2(rr[WAVE]);
                        i = wd & 255;
                        oc = (wd >> 8) & 255;
                        cA = (wd >> 16) & 255;
                        cB = wd >> 24;
                    } else {
                        i = L.cl[sl * NP2 + idx];
                        oc = ptype(L.S[i], L.S[i + dd]) * 25 + L.S[i + 1] * 5 + L.S[i + dd - 1];
                        cA = L.up[i + 1];
                        cB = L.dn[i + dd - 1];
                        mmo = L.dt[DT_MMI + oc];
                        mo = padd(L.ct[CT_ONEN + oc], mmo);
                    }
                    const int type = (oc * 41) >> 10;
                    const int si1 = (oc / 5) % 5;
                    const int sj1 = oc % 5;
                    const int uml = dd - 6 < 30 ? dd - 6 : 30;   // this lane's loop sizes
                    BCell C;
                    C.i = i + hb * (N - d + 2);
                    C.hb = hb;
                    C.ty8 = type * 8;
                    C.rs = uint32_t(r) * 4u;
                    C.ee = ae4 + uint32_t(r) * 4u;
                    C.r1 = (r & 1) != 0;
                    C.r2 = (r & 2) != 0;
                    C.eb = r & 1;
                    C.ea = sh == 2 ? ((r & 1) ? -(r >> 1) : (r >> 1)) : ((r & 1) ? -1 : 1);
                    C.ctb = (r & 2) ? CT_ONEN : CT_BUL;
                    C.A = cA;
                    C.B = cB;
                    const u32 tau = type > 2 ? tauE : 0u;
                    // the loop sizes' table energies only on the wave whose block reads them
                    // (bits of a literal: a runtime-indexed table would be a scalar load)
                    auto has = [&](unsigned bits) { return ((bits >> (sh * 8 + blk)) & 1u) != 0; };
                    C.m23f = has(size_bits(5)) ? padd(L.ct[CT_M23O + oc], fsm5) : INF16;
                    C.t11 = C.t12 = C.t21 = C.t22 = INF16;
                    {   // 1x1..2x2 energies from HBM (L2), used at the block end
                        const int ty8 = type * 8;
                        if (has(size_bits(2)) && uml >= 2) {
                            const int c2 = L.cc[off(dd - 4, N) + i + 1];
                            C.t11 = T11[((ty8 + ((c2 * 41) >> 10)) * 5 + si1) * 5 + sj1];
                        }
                        if (has(size_bits(3)) && uml >= 3) {
                            const int o3 = off(dd - 5, N) + i;
                            const int a2 = L.cc[o3 + 1], b2 = L.cc[o3 + 2];
                            const int ta = (a2 * 41) >> 10, tb = (b2 * 41) >> 10;
                            C.t12 = T21[(((ty8 + ta) * 5 + si1) * 5 + (a2 / 5) % 5) * 5 + sj1];
                            C.t21 = T21[(((tb * 8 + type) * 5 + (b2 / 5) % 5) * 5 + si1) * 5 + b2 % 5];
                        }
                        if (has(size_bits(4)) && uml >= 4) {
                            const int c2 = L.cc[off(dd - 6, N) + i + 2];
                            const int t2 = (c2 * 41) >> 10;
                            C.t22 = T22[((((ty8 + t2) * 5 + si1) * 5 + c2 % 5) * 5 + (c2 / 5) % 5) * 5 + sj1];
                        }
                    }
                    Acc a{INF16, INF16, INF16, INF16, INF16, INF16};
                    const bool mk = constrained && __ballot(C.A < uml || C.B < uml) != 0;
                    U.mk = mk;
                    PSTAMP(9);
                    if (sh == 2) mfe_block_s4(blk, U, C, a);
                    else if (sh == 1) mfe_block_s2(blk, U, C, a);
                    else mfe_block(blk, U, C, a);
                    PSTAMP(10);
                    u32 acc = pmin(pmin(a.s, padd(pmin(a.g0, a.g1), mmo)), pmin(padd(a.b, tau), padd(a.n, mo)));
                    if (sh == 2) acc = pmin(acc, padd(a.e, C.r2 ? mo : tau));
                    if (sh == 2) acc = fold_rows16(acc);
                    if (sh >= 1) acc = fold_halves(acc);
                    if (r == 0) {
                        int *pp = L.part + (dd & 3) * 2 * NP + i;
#ifndef ADX_ABL_NOATOM
                        atomicMin(pp, sext_lo(acc));
                        atomicMin(pp + NP, sext_hi(acc));
#else   // diagnostic (results wrong): plain stores instead of the atomic minima
                        pp[0] = sext_lo(acc);
                        pp[NP] = sext_hi(acc);
#endif
                    }
                }
            }
        }
        cPP = nPP, cwd = nwd, cmm = nmm;
        PSTAMP(3);
        // ---------------- M: split parts of qm for spans d and d+1 (lanes = cells x
        // slices of the split points, mfe_cells.hip): min over t >= 5 of
        // qm(i, i+t-1) + qm1(i+t, j), written to the span's slot for F
#ifndef ADX_ABL_NOM
        if (wid == mw[0] || wid == mw[1]) {
#else   // diagnostic (results wrong): no split parts
        if (false) {
#endif
            __builtin_amdgcn_s_setprio(PRIO_ROLE);
            {
                const int s = wid == mw[0] ? d : d + 1;
                if (s >= 9 && s <= N - 3) {   // no split point below span 9
                const int lo = qlo(s), hi = qhi(s);
                const int Lm = lanesets(hi - lo + 1);
                const int Tt = s - 4;
                u32 *slot = L.mla + (s % 6) * NP;
                for (int ls = 0; ls < Lm; ls++) {
                    const int nc = min(WAVE, hi - lo + 1 - ls * WAVE);
                    const int lc = nc <= 1 ? 0 : 32 - __clz(nc - 1);
                    const int cst = 1 << lc, lsl = 6 - lc;
                    const int c = lane & (cst - 1), rr = lane >> lc;
                    int i = lo + ls * WAVE + c;
                    const bool valid = c < nc;
                    if (!valid) i = hi;
                    const int j = i + s;
                    const int nb = Tt - 4;                                  // split points t = 5..Tt
                    const int bs = nb > 0 ? (nb + (1 << lsl) - 1) >> lsl : 0;
                    u32 sp0 = INF16, sp1 = INF16;
                    // split points in chunks of 16 and a last chunk of 16, 8 or 4 (bs is
                    // uniform, so are the chunk shapes; round 5: +0.7 %, reads past a
                    // slice's end cost as much as the ones in it on the M waves)
                    auto chunk = [&](auto nconst, int t0) __attribute__((always_inline)) {
                        constexpr int NR = decltype(nconst)::value;
                        u32 av[NR], rv[NR];
                        const uint32_t pa = aqm1 + uint32_t(colb(j) + i - 1 + t0) * 4u;
                        const uint32_t pr = aqm + uint32_t(rowb(i, N) - 5 + t0) * 4u;
                        if constexpr (NR == 16) {
                            asm volatile(
                                    "ds_read_b32 %0, %32 offset:0\n"
                                    "ds_read_b32 %1, %32 offset:4\n"
                                    "ds_read_b32 %2, %32 offset:8\n"
                                    "ds_read_b32 %3, %32 offset:12\n"
                                    "ds_read_b32 %4, %32 offset:16\n"
                                    "ds_read_b32 %5, %32 offset:20\n"
                                    "ds_read_b32 %6, %32 offset:24\n"
                                    "ds_read_b32 %7, %32 offset:28\n"
                                    "ds_read_b32 %8, %32 offset:32\n"
                                    "ds_read_b32 %9, %32 offset:36\n"
                                    "ds_read_b32 %10, %32 offset:40\n"
                                    "ds_read_b32 %11, %32 offset:44\n"
                                    "ds_read_b32 %12, %32 offset:48\n"
                                    "ds_read_b32 %13, %32 offset:52\n"
                                    "ds_read_b32 %14, %32 offset:56\n"
                                    "ds_read_b32 %15, %32 offset:60\n"
                                    "ds_read_b32 %16, %33 offset:0\n"
                                    "ds_read_b32 %17, %33 offset:4\n"
                                    "ds_read_b32 %18, %33 offset:8\n"
                                    "ds_read_b32 %19, %33 offset:12\n"
                                    "ds_read_b32 %20, %33 offset:16\n"
                                    "ds_read_b32 %21, %33 offset:20\n"
                                    "ds_read_b32 %22, %33 offset:24\n"
                                    "ds_read_b32 %23, %33 offset:28\n"
                                    "ds_read_b32 %24, %33 offset:32\n"
                                    "ds_read_b32 %25, %33 offset:36\n"
                                    "ds_read_b32 %26, %33 offset:40\n"
                                    "ds_read_b32 %27, %33 offset:44\n"
                                    "ds_read_b32 %28, %33 offset:48\n"
                                    "ds_read_b32 %29, %33 offset:52\n"
                                    "ds_read_b32 %30, %33 offset:56\n"
                                    "ds_read_b32 %31, %33 offset:60\n"
                                "s_waitcnt lgkmcnt(0)"
                                : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]), "=&v"(av[6]), "=&v"(av[7]), "=&v"(av[8]), "=&v"(av[9]), "=&v"(av[10]), "=&v"(av[11]), "=&v"(av[12]), "=&v"(av[13]), "=&v"(av[14]), "=&v"(av[15]), "=&v"(rv[0]), "=&v"(rv[1]), "=&v"(rv[2]), "=&v"(rv[3]), "=&v"(rv[4]), "=&v"(rv[5]), "=&v"(rv[6]), "=&v"(rv[7]), "=&v"(rv[8]), "=&v"(rv[9]), "=&v"(rv[10]), "=&v"(rv[11]), "=&v"(rv[12]), "=&v"(rv[13]), "=&v"(rv[14]), "=&v"(rv[15])
                                : "v"(pa), "v"(pr)
                                : "memory");
                        } else if constexpr (NR == 4) {
                            asm volatile(
                                    "ds_read_b32 %0, %8 offset:0\n"
                                    "ds_read_b32 %1, %8 offset:4\n"
                                    "ds_read_b32 %2, %8 offset:8\n"
                                    "ds_read_b32 %3, %8 offset:12\n"
                                    "ds_read_b32 %4, %9 offset:0\n"
                                    "ds_read_b32 %5, %9 offset:4\n"
                                    "ds_read_b32 %6, %9 offset:8\n"
                                    "ds_read_b32 %7, %9 offset:12\n"
                                "s_waitcnt lgkmcnt(0)"
                                : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(rv[0]), "=&v"(rv[1]), "=&v"(rv[2]), "=&v"(rv[3])
                                : "v"(pa), "v"(pr)
                                : "memory");
                        } else {
                            asm volatile(
                                    "ds_read_b32 %0, %16 offset:0\n"
                                    "ds_read_b32 %1, %16 offset:4\n"
                                    "ds_read_b32 %2, %16 offset:8\n"
                                    "ds_read_b32 %3, %16 offset:12\n"
                                    "ds_read_b32 %4, %16 offset:16\n"
                                    "ds_read_b32 %5, %16 offset:20\n"
                                    "ds_read_b32 %6, %16 offset:24\n"
                                    "ds_read_b32 %7, %16 offset:28\n"
                                    "ds_read_b32 %8, %17 offset:0\n"
                                    "ds_read_b32 %9, %17 offset:4\n"
                                    "ds_read_b32 %10, %17 offset:8\n"
                                    "ds_read_b32 %11, %17 offset:12\n"
                                    "ds_read_b32 %12, %17 offset:16\n"
                                    "ds_read_b32 %13, %17 offset:20\n"
                                    "ds_read_b32 %14, %17 offset:24\n"
                                    "ds_read_b32 %15, %17 offset:28\n"
                                "s_waitcnt lgkmcnt(0)"
                                : "=&v"(av[0]), "=&v"(av[1]), "=&v"(av[2]), "=&v"(av[3]), "=&v"(av[4]), "=&v"(av[5]), "=&v"(av[6]), "=&v"(av[7]), "=&v"(rv[0]), "=&v"(rv[1]), "=&v"(rv[2]), "=&v"(rv[3]), "=&v"(rv[4]), "=&v"(rv[5]), "=&v"(rv[6]), "=&v"(rv[7])
                                : "v"(pa), "v"(pr)
                                : "memory");
                        }
                        // reads past this slice's end belong to the next slice (a split point
                        // counted twice leaves the minimum unchanged): only the row end Tt masks
                        const int lim = Tt - t0;
                        if (__ballot(lim < NR - 1) == 0) {
#pragma unroll
                            for (int k = 0; k < NR; k += 2) {
                                sp0 = pmin(sp0, padd(rv[k], av[k]));
                                sp1 = pmin(sp1, padd(rv[k + 1], av[k + 1]));
                            }
                        } else {
#pragma unroll
                            for (int k = 0; k < NR; k += 2) {
                                sp0 = pmin(sp0, padd(rv[k], k <= lim ? av[k] : INF16));
                                sp1 = pmin(sp1, padd(rv[k + 1], k + 1 <= lim ? av[k + 1] : INF16));
                            }
                        }
                    };
                    int t0 = 5 + rr * bs;
                    for (int ch = 0; ch < (bs >> 4); ch++, t0 += 16) chunk(std::integral_constant<int, 16>{}, t0);
                    const int rem = bs & 15;
                    if (rem > 8) chunk(std::integral_constant<int, 16>{}, t0);
                    else if (rem > 4) chunk(std::integral_constant<int, 8>{}, t0);
                    else if (rem > 0) chunk(std::integral_constant<int, 4>{}, t0);
                    u32 split = pmin(sp0, sp1);
                    for (int k = cst; k < WAVE; k <<= 1) split = pmin(split, u32(__shfl_xor(int(split), k, WAVE)));
                    if (valid && rr == 0) slot[i] = pfin(split);
                }
                }
            }
            __builtin_amdgcn_s_setprio(0);
        }
        PSTAMP(4);
        // ---------------- Q: q5[j] for j = d-3, d-2 (qbm spans <= d-3 are final)
        if (wid == Q_WAVE) {
            const int j0 = d - 3, j1 = d - 2;
            const bool w0 = j0 >= 5 && j0 <= N && (!incr || j0 >= m_lo - 1);
            const bool w1 = j1 >= 5 && j1 <= N && (!incr || j1 >= m_lo - 1);
            if (w0 || w1) {
                __builtin_amdgcn_s_setprio(PRIO_ROLE);
                // the last step of an odd N has j1 = N + 1 (w1 false): its chain reads
                // column N instead, so no read leaves the tables (the result is unused)
                const int j1r = j1 <= N ? j1 : N;
                const int s0 = L.S[j0], s1 = L.S[j1r];
                const int sp0 = (j0 < N) ? L.S[j0 + 1] : 5, sp1 = (j1r < N) ? L.S[j1r + 1] : 5;   // no dangle past N
                u32 acc0 = INF16, acc1 = INF16;
                for (int k0 = 1; k0 <= j1r - 4; k0 += WAVE) {
                    const int kk = k0 + lane;
                    const bool ok1 = kk <= j1r - 4, ok0 = kk <= j0 - 4;
                    const int k = ok1 ? kk : 1;
                    const int sk = L.S[k], skm = (k > 1) ? L.S[k - 1] : 5;
                    const u32 q5k = L.q5[k - 1];
                    const int ix1 = off(j1r - k, N) + k - 1;
                    const int ix0 = off(max(j0 - k, 4), N) + k - 1;
                    const u32 ex1 = L.dt[DT_EXT + ptype(sk, s1) * 36 + skm * 6 + sp1];
                    const u32 ex0 = L.dt[DT_EXT + ptype(sk, s0) * 36 + skm * 6 + sp0];
                    const u32 t1 = padd(padd(q5k, L.qbm[ix1]), padd(L.ct[CT_INVMM + L.cc[ix1]], ex1));
                    const u32 t0 = padd(padd(q5k, L.qbm[ix0]), padd(L.ct[CT_INVMM + L.cc[ix0]], ex0));
                    acc1 = pmin(acc1, ok1 ? t1 : INF16);
                    acc0 = pmin(acc0, ok0 ? t0 : INF16);
                }
                const u32 red0 = wave_min(acc0), red1 = wave_min(acc1);
                if (lane == 0) {
                    u32 q0 = L.q5[j0];   // restored (refold) or initial when not recomputed
                    if (w0) {
                        q0 = pfin(pmin((L.up[j0] >= 1) ? L.q5[j0 - 1] : INF16, red0));
                        L.q5[j0] = q0;
                    }
                    if (w1) L.q5[j1] = pfin(pmin((L.up[j1] >= 1) ? q0 : INF16, red1));
                }
                __builtin_amdgcn_s_setprio(0);
            }
        }
        PSTAMP(5);
        lds_barrier();
        PSTAMP(6);
        sl = sl1;
    }
#ifdef ADX_STAMP
    if (lane == 0 && wid < 16)
        for (int k = 0; k < 16; k++) atomicAdd(&g_stamps_p[wid][k], st_acc[k]);
#endif
}

// the fold's write-back and 16-bit range check (one copy for all waves)
template <int NT, int NM>
__device__ __forceinline__ void pair_finish(const KArgs &ka, const int *vs, const CP &L, const IncM &inc, u32 &z,
                                            bool &bad) {
    const int N = uni(ka.variants[vs[0]].N);
    const int tid = threadIdx.x;
    z = L.q5[N];
    if (inc.dst) {   // this fold's tables: the next proposal's unchanged cells
        const size_t C = size_t(ka.cells);
        u32 *dp = inc.dst;
        for (int k = tid; k < int(C); k += NT) {
            dp[k] = L.qbm[k];
            dp[C + k] = L.qm[k];
            dp[2 * C + k] = L.qm1[k];
        }
        for (int k = tid; k <= N; k += NT) dp[3 * C + k] = L.q5[k];
        const int C16 = (((N - 4) * (N - 3)) / 2 + 15) >> 4;
        for (int k = tid; k < C16; k += NT) inc.cc_dst[k] = reinterpret_cast<const uint4 *>(L.cc)[k];
    }
    bool low = false;
    const int C = ((N - 4) * (N - 3)) >> 1;
    auto chk = [&](u32 x) {
        const s16x2 q = sv(x);
        low |= mfe16_inexact(q);
    };
    for (int k = tid; k < C; k += NT) {
        chk(L.qbm[k]);
        chk(L.qm[k]);
        chk(L.qm1[k]);
    }
    for (int k = tid; k <= N; k += NT) chk(L.q5[k]);
    bad = block_or(L.flag + 1, low);
}

// the fold instance of wave w (one per wave: mfe_pair_fold's WID)
template <int NT, int NM, int... Ws>
__device__ __forceinline__ void pair_fold_wave(std::integer_sequence<int, Ws...>, int w, const KArgs &ka,
                                               const DevScaled *__restrict__ XS, const DevTables *__restrict__ TT,
                                               const int *vs, const CP &L, const IncM &inc, bool constrained,
                                               const unsigned long long *sst) {
    ((w == Ws ? (mfe_pair_fold<NT, NM, Ws>(ka, XS, TT, vs, L, inc, constrained, sst), 0) : 0), ...);
}

constexpr int MFE_WPE = (2 * NWV + 3) / 4;
template <int NT, int NM>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFE_WPE, MFE_WPE)))
mfe_pair_kernel(const KArgs ka, const DevScaled *__restrict__ XS, const DevTables *__restrict__ TT, const uint8_t *seqs,
                int W, float *gout, const int *mask) {
    // one workgroup per (walker, fold group), as mfe_cells_kernel
    const CP L = PLay<NM>::carve();
    const int ng = ka.n_groups2;
    const int wb = int(blockIdx.x) / ng, g = int(blockIdx.x) % ng;
    if (wb >= W) return;
    const WalkerRef wr = walker_ref(ka, mask, wb);   // heaviest refolds first
    if (!wr.on) return;
    const int w = wr.w;
    if (threadIdx.x < 2) L.flag[threadIdx.x] = 0;
    __syncthreads();
    const int vs[2] = {ka.groups2[2 * g], ka.groups2[2 * g + 1]};
    IncM inc{nullptr, nullptr, 0, 0, nullptr, nullptr};
    if (ka.tab) {
        const size_t Gf = inc_group_floats(ka.cells, ka.Nmax, 1);
        const int cur = wr.cur;
        float *base = ka.tab + size_t(w) * 2 * ka.tab_slot;
        inc.dst = reinterpret_cast<u32 *>(base + size_t(1 - cur) * ka.tab_slot + size_t(g) * Gf);
        const size_t cco = inc_cc_offset(ka.cells, ka.Nmax, ng, g);
        inc.cc_dst = reinterpret_cast<uint4 *>(base + size_t(1 - cur) * ka.tab_slot + cco);
        // a sibling group may clear tab_valid[w] on overflow while this one reads it:
        // either value is correct (an incremental refold equals a fold from scratch)
        if (wr.valid && wr.c0 >= 0) {
            const int lb = ka.variants[vs[0]].before_len;
            inc.src = reinterpret_cast<const u32 *>(base + size_t(cur) * ka.tab_slot + size_t(g) * Gf);
            inc.cc_src = reinterpret_cast<const uint4 *>(base + size_t(cur) * ka.tab_slot + cco);
            inc.m_lo = wr.c0 + 1 + lb;
            inc.m_hi = wr.c1 + 1 + lb;
        }
    }
    u32 z = INF16;
    bool bad = false;
    unsigned long long sst[7] = {0, 0, 0, 0, 0, 0, 0};
    const bool constrained = pair_setup<NT, NM>(ka, XS, TT, vs, seqs + size_t(w) * ka.Nraw, L, inc, sst);
    pair_fold_wave<NT, NM>(std::make_integer_sequence<int, NWV>{}, uni(int(threadIdx.x) / WAVE), ka, XS, TT, vs, L,
                           inc, constrained, sst);
    pair_finish<NT, NM>(ka, vs, L, inc, z, bad);
    if (threadIdx.x == 0) {
        const s16x2 q = sv(z);
        const int hv[2] = {q.x, q.y};
        for (int h = 0; h < 2; h++) {
            const double e = hv[h] >= 0x4000 ? double(INFINITY) : static_cast<double>(hv[h]) / 100.0;
            gout[size_t(w) * ka.n_variants + vs[h]] = static_cast<float>(e);
        }
        if (bad && ka.ovf) {
            ka.ovf[w] = 1;
            if (ka.tab) ka.tab_valid[w] = 0;
        }
    }
}

template <int NM>
static hipError_t launch_pair_nm(const KArgs &ka, const uint8_t *seqs, int W, float *gout, const int *mask,
                                 hipStream_t stream) {
    constexpr size_t lds = PLay<NM>::BYTES;
    auto k = mfe_pair_kernel<NWV * WAVE, NM>;
    static bool configured = false;
    if (!configured) {
        // the carve addresses LDS from 0 (lds_at): no static LDS may precede the block
        hipFuncAttributes fa;
        hipError_t e = hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(k));
        if (e != hipSuccess) return e;
        if (fa.sharedSizeBytes != 0) return hipErrorInvalidKernelFile;
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        if (std::getenv("ADX_OCC")) {   // diagnostic: resident workgroups per CU at this LDS size
            int nb = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(k), NWV * WAVE, lds);
            std::fprintf(stderr, "mfe_pair_kernel<%d>: %d waves, %zu B LDS, %d VGPRs, %d workgroups per CU\n", NM,
                         NWV, lds, fa.numRegs, nb);
        }
        configured = true;
    }
    hipLaunchKernelGGL(k, dim3(W * ka.n_groups2), dim3(NWV * WAVE), lds, stream, ka, ka.X, ka.T, seqs, W, gout, mask);
    return hipGetLastError();
}

}  // namespace

// The pair kernel covers folded lengths up to 100 (two 100-nt walkers per CU).
bool mfe_pair_covers(const KArgs &ka) { return ka.Nmax <= 100; }

hipError_t launch_mfe_pair(const KArgs &ka, const uint8_t *seqs, int W, float *gout, const int *mask,
                           hipStream_t stream) {
    static_assert(PLay<100>::BYTES <= 80 * 1024, "two 100-nt walkers per CU");
    if (ka.Nmax <= 64) return launch_pair_nm<64>(ka, seqs, W, gout, mask, stream);
    if (ka.Nmax <= 100) return launch_pair_nm<100>(ka, seqs, W, gout, mask, stream);
    return hipErrorInvalidValue;
}

}  // namespace adx

#ifdef ADX_STAMP
extern "C" int adx_debug_stamps_pair(unsigned long long *out, int reset) {  // [16][16]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(adx::g_stamps_p), sizeof(adx::g_stamps_p)) != hipSuccess) return 1;
    if (reset) {
        static unsigned long long z[16][16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(adx::g_stamps_p), z, sizeof(z)) != hipSuccess) return 2;
    }
    return 0;
}
#endif
