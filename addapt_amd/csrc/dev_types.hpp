// Structures shared by the host setup code and the gfx950 kernels.
//
// HBM layout (all read-only during a launch unless noted):
//   DevTables  -- FP32 Boltzmann factors of the energy model (~230 KB, L2
//                 resident; loaded per term by the fold kernels)
//   DevScaled  -- per-context quantities that fold in the pf scale sigma^k
//                 (interior-loop term list, hairpin/ML power tables, ...)
//   constraint blobs -- per (context, macrostate) 5 byte arrays of N+2
//   walker state (read/write): sequences W*N (codes 1..4), scores W (f64),
//                 mt19937 streams A and C (W * 2 * 625 u32), counters W*4.
#pragma once

#include <cstdint>

namespace adx {

constexpr int NMAX = 255;          // positions (u8 indices in LDS lists)
constexpr int MAX_VARIANTS = 64;
constexpr int MAX_TERMS = 64;
constexpr int MAX_SPECIAL_HP = 64;
constexpr int MAX_MOTIF = 96;
constexpr int MT_WORDS = 625;      // 624 state words + index

// Per-context factor table copied into LDS by every workgroup
// (DevScaled::ctab).  "code" = the inner-pair code of a DP cell (p,q):
// rtype(p,q)*25 + S[q+1]*5 + S[p-1] (< 200), stored per cell in LDS; qbm
// holds qb * mismatchI[code], so qb = qbm * CT_INVMM[code].
constexpr int CT_INVMM = 0;    // [code] 1 / exp(-mismatchI)
constexpr int CT_BUL = 200;    // [code] INVMM * TermAU factor of the inner pair (bulges n >= 2)
constexpr int CT_ONEN = 400;   // [code] INVMM * exp(-mismatch_interior_1n)
constexpr int CT_M23O = 600;   // [code] exp(-mismatch_interior_23)
constexpr int CT_STK = 800;    // [8][8] stack
constexpr int CT_FB = 864;     // [n]   bulge n: exp(-bulge[n]) * sigma^(n+2)
constexpr int CT_F1N = 896;    // [nl]  1 x nl: exp(-(interior[nl+1] + ninio)) * sigma^(nl+3)
constexpr int CT_FSM = 928;    // [0] s^2 [1] bulge1 s^3 [2] s^4 [3] s^5 [4] s^6 [5] 2x3 s^7 [6] exp(-TermAU)
constexpr int CT_ONE = 935;    // 1.0 (neutral second factor)
constexpr int CT_SIZE = 936;
// generic interior factors exp(-(interior[u] + ninio)) * sigma^(u+2) for
// u = 6..30, n1 = 2..28: DevScaled::fgen[(u - 6) * FG_ROW + n1 - 2]
constexpr int FG_ROW = 27;
constexpr int FG_SIZE = 25 * FG_ROW;

// Interior-loop term lists of one closing pair (i,j), ordered by loop size
// u = n1 + n2 so that the terms allowed at a span (u <= min(30, span-6)) are a
// prefix.  The kernel maps term t of a list to lane t % 64 of slot t / 64.
//   S list: every loop whose factor depends on the inner pair (stack, bulges,
//           1x1 / 1x2 / 2x1 / 2x2 tables, 2x3 mismatches, 1 x n loops), <= 121
//   G list: generic loops n1, n2 >= 2, u >= 6 (factor fgen, inner mismatch
//           folded into qbm), <= 375
constexpr int NS_MAX = 128;
constexpr int NG_MAX = 384;
enum TermKind : uint8_t { TK_STK = 0, TK_B1, TK_I11, TK_I12, TK_I21, TK_I22, TK_M23, TK_BUL, TK_1N };

// Fold modes.  Partition function (KArgs::mode 0): DevTables / DevScaled hold
// FP32 Boltzmann factors (with the pf scale sigma^k), "impossible" = 0.
// Minimum free energy (mode 1): the same layouts hold energies in dcal/mol
// (integers, exact in FP32), factor products become sums, sigma^k becomes 0,
// "impossible" = MFE_BIG (kernels.hip MinPlus).
constexpr float MFE_BIG = 1.0e7f;
constexpr float MFE_MARK = 3.0e7f;   // non-pairable cell mark of the MFE tables

struct DevTables {         // exp(-E/kT) (PF) or E (MFE), FP32; pair type 0 rows are "impossible"
    float stack[8][8];
    float mmH[8][5][5];
    float mmI[8][5][5];
    float mm1n[8][5][5];
    float mm23[8][5][5];
    float mlstem[8][5][5];   // mismatchM * TermAU * MLintern (dangles = 2)
    float ext[8][6][6];      // exterior stem; neighbour code 5 = absent
    float termAU[8];
    float int11[8][8][5][5];
    float int21[8][8][5][5][5];
    float int22[8][8][5][5][5][5];
};

struct DevScaled {
    float ctab[CT_SIZE];     // see CT_* (copied to LDS)
    float fgen[FG_SIZE];     // generic interior factors
    // MFE only (mfe_cells.hip): generic interior energy = il[u] + nin[|n1 - n2|]
    float il[32];            // interior[u]
    float nin[32];           // min(MAX_NINIO, k * ninio)
    // MFE packed (upload_mfe16) only, per loop size u: il[u] + nin[k] (k = 0..5),
    // bulge[u], 1 x (u-1) -- the interior-loop blocks' uniform energy record
    uint32_t ku16[32][8];
    // interior term lists (see NS_MAX); *_cnt[umax] = terms with u <= umax
    uint8_t s_n1[NS_MAX], s_n2[NS_MAX], s_kind[NS_MAX];
    float s_f[NS_MAX];       // constant factor (sigma power, bulge / 1xn length)
    uint8_t g_n1[NG_MAX], g_u[NG_MAX];
    float g_f[NG_MAX];
    int s_cnt[32], g_cnt[32];
    float sig[NMAX + 4];     // sigma^k
    float hp[NMAX + 1];      // hairpin length factor * sigma^(u+2)
    float pwml[NMAX + 1];    // (expMLbase * sigma)^t
    float mlclosing;         // expMLclosing * sigma^2
    float mlbase_sig;        // expMLbase * sigma
    int n_special;
    uint32_t sp_key[MAX_SPECIAL_HP];
    float sp_val[MAX_SPECIAL_HP];   // exp(-E_special) * sigma^(u+2)
    double log_sigma;
    double kT;               // kcal/mol
    // ligand motif (vrna_sc_add_hi_motif)
    int motif_len;
    uint8_t motif_code[MAX_MOTIF];
    int8_t motif_pt[MAX_MOTIF];     // partner offset or -1
    float motif_extra;              // exp(-Eint)(exp(-bonus)-1) * sigma^L
};

struct DevVariant {
    int N;            // folded length (context-padded)
    int before_len;   // context prefix length
    int ctx;          // context index (-1 none)
    int cons_off;     // byte offset of this variant's constraint arrays
    int motif;        // 1 = holo (ligand motif active)
    int pad;
};

struct DevTermMap {   // per (context, term)
    int vfree, vcons;
    int favorable;
    double weight;
    int kind;         // 0 = MacrostateProbTerm, 1 = base-pair probability term
    int pidx;         // kind 1: index into KArgs::pairs / the per-walker pair probabilities
};

// Special-hairpin key: 3 bits per base of the closing-pair-inclusive loop.
__host__ __device__ inline uint32_t hp_key(const uint8_t *S, int i, int len) {
    uint32_t k = static_cast<uint32_t>(len);
    for (int t = 0; t < len; t++) k = (k << 3) | S[i + t];
    return k;
}

// floats of one fold group's tables in the incremental-fold state: per value
// array qbm, qm, qm1 (cells each) and q5 (Nmax + 2)
__host__ __device__ inline size_t inc_group_floats(int cells, int Nmax, int P) {
    return size_t(P) * (3 * size_t(cells) + size_t(Nmax) + 2);
}
// MFE (packed 16-bit) slots also keep every cell's inner-pair code (one byte per
// cell, 16-byte aligned, after the n_groups2 groups' value arrays), so a refold
// restores the codes with the tables and recomputes only its band's
// (mfe_pair.hip; every MFE16 kernel writes them)
__host__ __device__ inline size_t inc_cc_floats(int cells) { return (size_t(cells) + 15) / 16 * 4; }
__host__ __device__ inline size_t inc_cc_offset(int cells, int Nmax, int n_groups2, int g) {
    return (size_t(n_groups2) * inc_group_floats(cells, Nmax, 1) + 3) / 4 * 4 + size_t(g) * inc_cc_floats(cells);
}
// the same for the PF slots (two value arrays per group: pf_cells.hip, kernels.hip SumProd)
__host__ __device__ inline size_t inc_cc_offset_pf(int cells, int Nmax, int n_groups2, int g) {
    return (size_t(n_groups2) * inc_group_floats(cells, Nmax, 2) + 3) / 4 * 4 + size_t(g) * inc_cc_floats(cells);
}

struct KArgs {
    const DevTables *T;
    const DevScaled *X;
    const DevVariant *variants;
    const uint8_t *cons;        // constraint blobs
    const uint8_t *ctx_seq;     // concatenated before/after context codes
    const int *ctx_off;         // per context: before offset, before len, after offset, after len
    const DevTermMap *tmap;     // [n_ctx_eff * n_terms]
    int n_variants;
    int n_terms;
    int n_ctx_eff;              // max(1, contexts)
    int Nraw;                   // raw device length
    int Nmax;                   // max folded length over variants
    int cells;                  // (Nmax-4)(Nmax-3)/2
    const int *groups2;         // [n_groups2][2]: variants folded in lockstep (apo, holo of one
    int n_groups2;              //   (context, macrostate); a lone variant is paired with itself)
    int opt;                    // launch-time LDS options (kernels.hip choose_opt)
    int mode;                   // 0 = partition functions, 1 = minimum free energies (MinPlus tables)
    // base-pair probabilities (outside pass, bppm_kernel)
    const int *bvars;           // [n_bvars] variants folded with an outside pass
    int n_bvars;
    const int *bvar_slot;       // [n_bvars] the variant's tables in the groups2 slot layout
                                //   (2 * group + half; host-computed, adx_api.cpp upload_all)
    const int *pairs;           // [n_pairs][3]: bvars index, i, j (1-based, folded coordinates)
    int n_pairs;
    const double *pair_p;       // [W][n_pairs] probabilities written by bppm_kernel (score input)
    char *bppm_scratch;         // global outside tables when they do not fit LDS (N >~ 110)
    // MFE: packed 16-bit tables (two variants per value) and the per-walker flag of
    // folds that left the 16-bit exact range (re-folded with the FP32 tables T, X)
    const DevTables *T16;
    const DevScaled *X16;
    int *ovf;
    int mfe_cells_ok;           // the lanes = cells MFE kernel covers this energy model (mfe_cells.hip)
    // incremental folds (kernels.hip Inc): per walker two slots of every group's
    // tables (tab_slot floats each), the current slot and whether it is valid,
    // and the hull of the positions the step's proposal changed (-1: none)
    float *tab;
    size_t tab_slot;
    uint8_t *cur_slot;
    uint8_t *tab_valid;
    const int *chg;
    // PF folds longer than pf_cells covers (pf_ring.hip): one workgroup per
    // variant, qb in a ring of diagonals; the slot's qm / qm1 are then
    // diagonal-major (decided once per context: every kernel reading the slot
    // must agree).  ring_scratch: qb of stateless launches (W * 2 * n_groups2 * cells)
    int pf_ring;
    float *ring_scratch;
    // [W][n_variants] per-variant energies of the step's proposals when the score
    // waits for the outside pass (pair terms): score_kernel -> bppm_kernel
    // (re-using the inside tables just written) -> combine_kernel
    float *gstep;
    // MC steps: the walkers in launch order, heaviest refold first, so the long
    // folds do not trail the launch (kernels.hip order_kernel, from the weight
    // classes in ocls); the fold kernels map blockIdx through it
    // (fold_common.hpp walker_at); null: blockIdx order
    int *order;
    const uint8_t *ocls;
    // MC steps: the scores a fold launch leaves as per-variant energies in gstep
    // are combined by the step's tail (kernels.hip accept_walker), not by a
    // combine_kernel launch of their own
    int defer_comb;
};

// Monte Carlo state (device, read/write).
struct StepArgs {
    uint8_t *cur_seq;           // W * Nraw codes
    double *cur_score;          // W
    uint32_t *mtA, *mtC;        // W * MT_WORDS
    int64_t *counters;          // W * 4
    double *last_diff;          // W (score_diff carried across steps)
    double *auto_T;             // W
    double *train;              // W * period
    int *ntrain;                // W
    int *err;                   // W (0 ok, else move error code)
    uint8_t *prop_seq;          // W * Nraw proposal
    double *prop_score;         // W
    int *changed;               // W (1 = scored this step)
    int *pick, *bcode;          // W
    double *temp, *u;           // W
    int Nraw;
    const int *mut;             // freely mutable positions (0-based raw), M
    const int *clo_off;         // M + 1
    const int *clo_pos;         // closure positions (0-based raw)
    const uint8_t *clo_par;     // 0 same base, 1 complement
    const int *clo_err;         // M
    int M;
    int thermo_kind;
    double t_fixed, t_hi, t_lo;
    int cycle_len;
    double ln_target_rate;   // log(target rate), host libm (the reference divides by log(rate), sampling.cc:395)
    int period;
    long long step0;            // global step index of the first step of this launch
    int nsteps;
    int W;
    // optional trace (nullptr when off), step-major [s * W + w]
    int32_t *tr_pos;
    int8_t *tr_base;
    int32_t *tr_outcome;
    double *tr_temp, *tr_prop, *tr_cur, *tr_u;
    double *tr_terms;           // [(s*W + w) * n_terms_total]
    int *chg;                   // W * 2: hull of the positions the proposal changed (-1: none)
    // the weight class of the proposal's fold (KArgs::ocls; null: none), the
    // incremental-fold state accept updates and the MFE overflow flags a
    // proposal clears (null when absent)
    uint8_t *cls;
    uint8_t *cur_slot, *tab_valid;
    int *ovf;
};

}  // namespace adx
