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
#include <cstdlib>
#include <cstring>

#include "dev_types.hpp"
#include "fold_common.hpp"

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


// ---------------------------------------------------------------- semirings
// One kernel body folds both energy models:
//   SumProd  McCaskill partition function: FP32 Boltzmann factors with the pf
//            scale sigma (vrna_pf);
//   MinPlus  Zuker minimum free energy: integer dcal/mol held in FP32 (exact
//            below 2^24), "impossible" = BIG and above (never +inf, so 0/1
//            selector products stay finite), the same loop decomposition with
//            sums of energies in place of products of factors.
// The non-pairable cell mark (a value a finished cell never takes) is -0.0f
// for SumProd and MARK for MinPlus.
struct SumProd {
    static constexpr bool MFE = false;
    static constexpr int NV = 1;   // variants per value
    __device__ static float zero() { return 0.f; }
    __device__ static float one() { return 1.f; }
    __device__ static float add(float a, float b) { return a + b; }
    __device__ static float mul(float a, float b) { return a * b; }
    __device__ static float fma(float a, float b, float c) { return fmaf(a, b, c); }
    __device__ static float mark() { return -0.0f; }
    __device__ static bool is_mark(float x) { return __float_as_uint(x) == 0x80000000u; }
    __device__ static float fin(float x) { return x + 0.0f; }   // never -0
};
struct MinPlus {
    static constexpr bool MFE = true;
    static constexpr int NV = 1;
    __device__ static float zero() { return MFE_BIG; }
    __device__ static float one() { return 0.f; }
    __device__ static float add(float a, float b) { return fminf(a, b); }
    __device__ static float mul(float a, float b) { return a + b; }
    __device__ static float fma(float a, float b, float c) { return fminf(a + b, c); }
    __device__ static float mark() { return MFE_MARK; }
    __device__ static bool is_mark(float x) { return x == MFE_MARK; }
    __device__ static float fin(float x) { return fminf(x, MFE_BIG); }   // never MARK
};

// Packed 16-bit min-plus: TWO variants per 32-bit value (the apo and holo folds
// of one group in the low / high half), v_pk_add_i16 (saturating) and
// v_pk_min_i16, so one instruction advances both folds and the tables take
// half the LDS of the FP32 pair.  Values travel in float registers as raw bits
// (only moves, selects and these ops touch them).  Encoding per half: integer
// dcal/mol; 0x7FFF = impossible; any value >= 0x4000 counts as impossible and
// is reset to 0x7FFF when a cell is stored (fin).  Exact while every stored
// value stays >= MFE16_FLOOR (checked at the end of the fold; a walker that
// fails the check is re-folded by the FP32 MinPlus kernel).
struct MinPlus16 {
    static constexpr bool MFE = true;
    static constexpr int NV = 2;
    __device__ static s16x2 v(float x) { return __builtin_bit_cast(s16x2, x); }
    __device__ static float f(s16x2 x) { return __builtin_bit_cast(float, x); }
    __device__ static float zero() { return __uint_as_float(0x7FFF7FFFu); }
    __device__ static float one() { return 0.f; }
    __device__ static float add(float a, float b) { return f(__builtin_elementwise_min(v(a), v(b))); }
    __device__ static float mul(float a, float b) { return f(__builtin_elementwise_add_sat(v(a), v(b))); }
    __device__ static float fma(float a, float b, float c) { return add(mul(a, b), c); }
    __device__ static float mark() { return __uint_as_float(0x7FFE7FFEu); }
    __device__ static bool is_mark(float x) { return __float_as_uint(x) == 0x7FFE7FFEu; }
    __device__ static float fin(float x) {   // halves in [0x4000, 0x7FFF] -> 0x7FFF
        const uint32_t u = __float_as_uint(x);
        const uint32_t imp = (u & ~(u >> 1)) & 0x40004000u;
        return __uint_as_float(u | ((imp >> 14) * 0x7FFFu));
    }
};

// Loop-factor selectors of qb_terms (0/1 selector floats from the term lists):
// the outer-pair factor of a slot-0 term, the prefetched table factor, and the
// slot-1 choice between the 1xn and bulge outer factor.
template <class SR>
__device__ __forceinline__ float sel_outer(float eb, float em, float e3, float tau, float mo, float m23) {
    if constexpr (SR::NV == 2)
        return eb != 0.f ? tau : (em != 0.f ? mo : (e3 != 0.f ? m23 : SR::one()));
    const float one = SR::one();
    return fmaf(eb, tau - one, fmaf(em, mo - one, fmaf(e3, m23 - one, one)));
}
template <class SR>
__device__ __forceinline__ float sel_tab(float eg, float gtab) {
    if constexpr (SR::NV == 2) return eg != 0.f ? gtab : SR::one();
    return fmaf(eg, gtab - SR::one(), SR::one());
}
template <class SR>
__device__ __forceinline__ float sel2(float em1, float mo, float tau) {
    if constexpr (SR::NV == 2) return em1 != 0.f ? mo : tau;
    return fmaf(em1, mo - tau, tau);
}

// Full-wave reductions via DPP (quad_perm, row_shr, row_bcast): VALU-only, no
// LDS crossbar.  Lanes a DPP move does not write keep the identity (SR::zero).
template <class SR, int CTRL, int ROWS>
__device__ __forceinline__ float dpp_op(float v) {
    const int moved = __builtin_amdgcn_update_dpp(__float_as_int(SR::zero()), __float_as_int(v), CTRL, ROWS,
                                                  0xf, false);
    return SR::add(v, __int_as_float(moved));
}
// Reduction over each row of 16 lanes; the row total lands in lane 15 of the row.
template <class SR = SumProd>
__device__ __forceinline__ float row_sum(float v) {
    v = dpp_op<SR, 0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_op<SR, 0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_op<SR, 0x114, 0xf>(v);  // row_shr:4
    v = dpp_op<SR, 0x118, 0xf>(v);  // row_shr:8
    return v;
}
template <class SR = SumProd>
__device__ __forceinline__ float wave_sum(float v) {
    v = dpp_op<SR, 0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_op<SR, 0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_op<SR, 0x114, 0xf>(v);  // row_shr:4
    v = dpp_op<SR, 0x118, 0xf>(v);  // row_shr:8
    v = dpp_op<SR, 0x142, 0xa>(v);  // row_bcast:15
    v = dpp_op<SR, 0x143, 0xc>(v);  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}



constexpr int CHUNK = 16;      // closing-pair cells per chunk of one wave (4 prefetch lanes each)
constexpr int GSLOTS = NG_MAX / WAVE;   // 6
constexpr int SSLOTS = NS_MAX / WAVE;   // 2
constexpr int LDS_LIMIT = 160 * 1024;
constexpr int MAXLOOP_K = 30;  // largest interior loop (ViennaRNA MAXLOOP)

// LDS carve-out for one workgroup folding P variants in lockstep (P = 2: the
// apo and holo folds of one (context, macrostate), which share every cell,
// pair type and loop factor and differ only by the ligand-motif bonus).
// lds_layout() is the single source of the layout: the kernel carves with it
// and the host sizes the launch with it.
template <int P>
struct Lds {
    float *qbm[P], *qm[P], *qm1[P];
    float *mla[P];     // [2][np] per variant: sum_k qm[i][k-1] qm1[k][j] of the last two qm diagonals
    float *q5[P];
    uint8_t *cc;       // inner-pair code per cell (diagonal-major), shared
    uint8_t *pcnt;     // [d] pairable cells of diagonal d, shared
    uint8_t *wsc;      // without rec: [wave][64] i of the cells of a wave's chunk
    uint8_t *rec;      // optional (null when it does not fit): i of every pairable cell, by
                       //   diagonal and rank
    uint32_t *rec32;   // optional, instead of rec when it fits: the full record word
                       //   i | oc << 8 | up[i+1] << 16 | dn[j-1] << 24 (see load_chunk)
    uint16_t *rbase;   // with rec: first record of diagonal d
    uint32_t *rt;      // optional: rt[d * NW + w] = kb_lo | kb_hi << 8 | km_lo << 16 | km_hi << 24
    float *ct;         // CT_SIZE factor table (DevScaled::ctab)
    float *dt;         // per-cell tables (DT_*)
    uint16_t *gd;      // G list: n1 | n2 << 8        (NG_MAX)
    float *gf;         // G list factors               (NG_MAX)
    uint32_t *sd;      // S list: n1 | n2 << 8 | kind << 16 (NS_MAX)
    float *sf;         // S list factors               (NS_MAX)
    float *pw;         // (expMLbase sigma)^t          (Nmax + 1)
    double *G;         // per-variant ensemble energies
    uint8_t *S, *up, *dn, *ptn, *enc, *flg, *mat, *raw;
    int np;
};

// DRY = true: sizes only (host); false: carve `base` (device; no null test, so
// the pointers stay in the LDS address space)
template <bool DRY, int P>
__host__ __device__ inline size_t lds_layout(char *base, int cells, int Nmax, int nvar, Lds<P> *L,
                                             int pl_mode = 0, bool with_rt = false, int nw = 16) {
    // pl_mode: 0 no record array, 1 rec (bytes), 2 rec32 (words)
    size_t o = 0;
    auto take = [&](size_t bytes) -> char * {
        char *p = DRY ? nullptr : base + o;
        o += (bytes + 15) & ~size_t(15);
        return p;
    };
    const size_t C = size_t(cells);
    const int NP = Nmax + 2;
    Lds<P> l;
    for (int p = 0; p < P; p++) {
        l.qbm[p] = reinterpret_cast<float *>(take(C * 4));
        l.qm[p] = reinterpret_cast<float *>(take(C * 4));
        l.qm1[p] = reinterpret_cast<float *>(take(C * 4));
        l.mla[p] = reinterpret_cast<float *>(take(2 * NP * 4));
        l.q5[p] = reinterpret_cast<float *>(take(NP * 4));
    }
    l.cc = reinterpret_cast<uint8_t *>(take(C));
    l.pcnt = reinterpret_cast<uint8_t *>(take(NP));
    l.wsc = pl_mode ? nullptr : reinterpret_cast<uint8_t *>(take(16 * WAVE));
    l.ct = reinterpret_cast<float *>(take(CT_SIZE * 4));
    l.dt = reinterpret_cast<float *>(take(size_t(DT_HP + Nmax + 1) * 4));
    l.gd = reinterpret_cast<uint16_t *>(take(NG_MAX * 2));
    l.gf = reinterpret_cast<float *>(take(NG_MAX * 4));
    l.sd = reinterpret_cast<uint32_t *>(take(NS_MAX * 4));
    l.sf = reinterpret_cast<float *>(take(NS_MAX * 4));
    l.pw = reinterpret_cast<float *>(take(size_t(Nmax + 1) * 4));
    l.G = reinterpret_cast<double *>(take(size_t(nvar) * 8));
    l.S = reinterpret_cast<uint8_t *>(take(NP));
    l.up = reinterpret_cast<uint8_t *>(take(NP));
    l.dn = reinterpret_cast<uint8_t *>(take(NP));
    l.ptn = reinterpret_cast<uint8_t *>(take(NP));
    l.enc = reinterpret_cast<uint8_t *>(take(NP));
    l.flg = reinterpret_cast<uint8_t *>(take(NP));
    l.mat = reinterpret_cast<uint8_t *>(take(NP));
    l.raw = reinterpret_cast<uint8_t *>(take(NP));
    // pairable cells (i, j), j - i >= 4: S[i] and S[j] sit on opposite sides of the
    // bipartite pairing graph {A,G} x {C,U}, so there are at most N^2/4 of them
    const size_t nrec = size_t(Nmax) * Nmax / 4 + Nmax;
    l.rec = pl_mode == 1 ? reinterpret_cast<uint8_t *>(take(nrec)) : nullptr;
    l.rec32 = pl_mode == 2 ? reinterpret_cast<uint32_t *>(take(nrec * 4)) : nullptr;
    l.rbase = pl_mode ? reinterpret_cast<uint16_t *>(take(size_t(NP) * 2)) : nullptr;
    l.rt = with_rt ? reinterpret_cast<uint32_t *>(take(size_t(NP) * nw * 4)) : nullptr;
    l.np = NP;
    if (!DRY) *L = l;
    return o;
}

template <int P>
__device__ void load_ctab(const KArgs &ka, const Lds<P> &L) {
    const int NT = blockDim.x;
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
    for (int k = threadIdx.x; k <= ka.Nmax; k += NT) {
        L.dt[DT_HP + k] = X.hp[k];
        L.pw[k] = X.pwml[k];
    }
    for (int k = threadIdx.x; k < NG_MAX; k += NT) {
        L.gd[k] = static_cast<uint16_t>(X.g_n1[k] | ((X.g_u[k] - X.g_n1[k]) << 8));
        L.gf[k] = X.g_f[k];
    }
    for (int k = threadIdx.x; k < NS_MAX; k += NT) {
        L.sd[k] = uint32_t(X.s_n1[k]) | (uint32_t(X.s_n2[k]) << 8) | (uint32_t(X.s_kind[k]) << 16);
        L.sf[k] = X.s_f[k];
    }
}

// ---------------------------------------------------------------- hard constraints
// flg bits: 1 = 'x' (no pair), 2 = '<' (pairs upstream), 4 = '>' (downstream);
// ptn = enforced partner (0 none); enc = innermost enclosing enforced pair id.
template <int P>
__device__ __forceinline__ bool allowed(const Lds<P> &L, int i, int j) {
    const int fi = L.flg[i], fj = L.flg[j];
    if ((fi | fj) & 1) return false;
    if ((fi & 2) || (fj & 4)) return false;
    const int pi = L.ptn[i], pj = L.ptn[j];
    if (pi) return pi == j;
    if (pj) return pj == i;
    return L.enc[i] == L.enc[j];
}

// ceil(x / y) for 0 < y, |x| < 2^22 (uniform operands; float reciprocal + exact fix-up,
// the scalar unit has no integer divide)
__device__ __forceinline__ int cdiv_pos(int x, int y) {
    if (x <= 0) return 0;
    int q = static_cast<int>(static_cast<float>(x) * __builtin_amdgcn_rcpf(static_cast<float>(y)));
    if (q * y < x) q++;
    if (q * y < x) q++;
    if ((q - 1) * y >= x) q--;
    return uni(q);
}
__device__ __forceinline__ int clampi(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

// Reductions of two per-lane values over the wave: permlane32 swap folds the
// halves (lanes 0-31 then carry a, 32-63 carry b), one row/half DPP chain finishes.
template <class SR>
__device__ __forceinline__ void wave_sum2(float a, float b, float &sa, float &sb) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    float v = SR::add(__uint_as_float(r[0]), __uint_as_float(r[1]));
    v = dpp_op<SR, 0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_op<SR, 0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_op<SR, 0x114, 0xf>(v);  // row_shr:4
    v = dpp_op<SR, 0x118, 0xf>(v);  // row_shr:8
    v = dpp_op<SR, 0x142, 0xa>(v);  // row_bcast:15 -> lane 31 = red(a), lane 63 = red(b)
    sa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 31));
    sb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

template <class SR, int P>
__device__ __forceinline__ void wave_sums(const float (&v)[P], float (&s)[P]) {
    if constexpr (P == 2) wave_sum2<SR>(v[0], v[1], s[0], s[1]);
    else s[0] = wave_sum<SR>(v[0]);
}

// ---------------------------------------------------------------- closing-pair terms
// Per-lane descriptors of one span's interior-loop terms (lane t of slot s =
// term s*64 + t of the S / G lists, dev_types.hpp).  Invalid lanes carry offset
// 0 (a finished cell) and factor SR::zero().
struct TermLanes {
    int offG[GSLOTS];      // qbm index of the inner cell minus i
    float fG[GSLOTS];
    int offS[SSLOTS];
    float fS[SSLOTS];
    int b1[SSLOTS];        // ct base of the inner-pair factor (INVMM / BUL / ONEN)
    int b2;                // slot 0: ct base of the second factor (STK / M23O / ONE)
    int mwt, mwc;          // slot 0: all-ones masks adding ty*8+t2 (stack) / code (2x3)
    float eb, em, e3, eg;  // slot 0: 0/1 selectors of tau, mo, m23 and the table factor
    float em1;             // slot 1: 1 = 1xn (mo), 0 = bulge (tau)
    int gsel;              // slot 0: which prefetched table factor (kind - TK_I11) & 3
};

// Uniform data of one closing pair (i, j) of the current span.
struct CellU {
    int i, ty8, A, B;
    float mmo, tau, mo, m23;
};

// Interior-loop sums of (i, j) for the P variants (the outer mismatch of the
// generic loops applied here): SS / SG slots, MK = constrained cell.  Every
// loop factor is computed once and applied to the P tables.
template <class SR, int SS, int SG, bool MK, int P>
__device__ __forceinline__ void qb_terms(const Lds<P> &L, const TermLanes &D, const CellU &u, float gtab,
                                         float (&out)[P]) {
    if (SS == 0) {
#pragma unroll
        for (int p = 0; p < P; p++) out[p] = SR::zero();
        return;
    }
    const float *ct = L.ct;
    const int lane = threadIdx.x & (WAVE - 1);
    float q[P][SG > 0 ? SG : 1];
#pragma unroll
    for (int s = 0; s < SG; s++)
#pragma unroll
        for (int p = 0; p < P; p++) q[p][s] = L.qbm[p][D.offG[s] + u.i];
    const int ix0 = D.offS[0] + u.i;
    float qs0[P], qs1[P];
#pragma unroll
    for (int p = 0; p < P; p++) qs0[p] = L.qbm[p][ix0];
    const int c0 = L.cc[ix0];
    int c1 = 0;
    if (SS > 1) {
        const int ix1 = D.offS[1] + u.i;
#pragma unroll
        for (int p = 0; p < P; p++) qs1[p] = L.qbm[p][ix1];
        c1 = L.cc[ix1];
    }
    float fg[SG > 0 ? SG : 1];
#pragma unroll
    for (int s = 0; s < SG; s++) {
        float f = D.fG[s];
        if (MK) {   // constrained cell: n1 <= A and n2 <= B (descriptor re-read from LDS)
            const int pk = L.gd[s * WAVE + lane];
            f = ((pk & 255) <= u.A && (pk >> 8) <= u.B) ? f : SR::zero();
        }
        fg[s] = f;
    }
    // slot 0: stack / bulge 1 / 1x1..2x2 tables / 2x3 / bulges / 1xn.  uf and gf
    // select (0/1 selectors, one per kind) the outer-pair factor and the
    // prefetched table factor, or the semiring one.
    const int t2 = (c0 * 41) >> 10;
    const int i2 = D.b2 + ((u.ty8 + t2) & D.mwt) + (c0 & D.mwc);
    const float uf = sel_outer<SR>(D.eb, D.em, D.e3, u.tau, u.mo, u.m23);
    const float gf = sel_tab<SR>(D.eg, gtab);
    float f0 = SR::mul(SR::mul(SR::mul(ct[D.b1[0] + c0], ct[i2]), SR::mul(D.fS[0], uf)), gf);
    if (MK) {
        const int pk = int(L.sd[lane]);
        f0 = ((pk & 255) <= u.A && ((pk >> 8) & 255) <= u.B) ? f0 : SR::zero();
    }
    float f1 = SR::zero();
    if (SS > 1) {
        // slot 1: bulges and 1xn only
        f1 = SR::mul(ct[D.b1[1] + c1], SR::mul(D.fS[1], sel2<SR>(D.em1, u.mo, u.tau)));
        if (MK) {
            const int pk = int(L.sd[WAVE + lane]);
            f1 = ((pk & 255) <= u.A && ((pk >> 8) & 255) <= u.B) ? f1 : SR::zero();
        }
    }
#pragma unroll
    for (int p = 0; p < P; p++) {
        float g0 = SR::zero(), g1 = SR::zero();
#pragma unroll
        for (int s = 0; s < SG; s++) {
            if (s & 1) g1 = SR::fma(q[p][s], fg[s], g1);
            else g0 = SR::fma(q[p][s], fg[s], g0);
        }
        float sa = SR::mul(qs0[p], f0);
        if (SS > 1) sa = SR::fma(qs1[p], f1, sa);
        out[p] = SR::fma(SR::add(g0, g1), u.mmo, sa);
    }
}

template <class SR, bool MK, int P>
__device__ __forceinline__ void qb_terms_dispatch(int sS, int sG, const Lds<P> &L, const TermLanes &D,
                                                  const CellU &u, float gtab, float (&out)[P]) {
    if (sS == 2) {
        switch (sG) {
            case 6: qb_terms<SR, 2, 6, MK, P>(L, D, u, gtab, out); return;
            case 5: qb_terms<SR, 2, 5, MK, P>(L, D, u, gtab, out); return;
            case 4: qb_terms<SR, 2, 4, MK, P>(L, D, u, gtab, out); return;
            case 3: qb_terms<SR, 2, 3, MK, P>(L, D, u, gtab, out); return;
            default: qb_terms<SR, 2, 2, MK, P>(L, D, u, gtab, out); return;
        }
    }
    if (sS == 1) {
        switch (sG) {
            case 0: qb_terms<SR, 1, 0, MK, P>(L, D, u, gtab, out); return;
            case 1: qb_terms<SR, 1, 1, MK, P>(L, D, u, gtab, out); return;
            default: qb_terms<SR, 1, 2, MK, P>(L, D, u, gtab, out); return;
        }
    }
    qb_terms<SR, 0, 0, MK, P>(L, D, u, gtab, out);
}

// ---------------------------------------------------------------- work split
// Per-diagonal item counts and estimated costs of iteration d (units ~8 cycles).
#ifndef ADX_CA0
#define ADX_CA0 50
#endif
#ifndef ADX_CB1
#define ADX_CB1 16
#endif
#ifndef ADX_CB0
#define ADX_CB0 16
#endif
struct RangeCost {
    int cp, cq, umax, nS, nG, sS, sG, nit, sQ5, cqg, ca, cb, c5, Ct;
};

template <int P>
__host__ __device__ inline RangeCost range_cost(int d, int N, int cp, int cq) {
    RangeCost r;
    const int sq = d - 1;                                   // qm span
    r.cp = cp;
    r.cq = cq;                                              // qm cells of span sq to fold
    r.umax = d - 6 < 30 ? d - 6 : 30;
    // |S|, |G| of the terms with u <= umax (dev_types.hpp lists, closed form)
    r.nS = r.umax < 0 ? 0 : r.umax <= 5 ? ((r.umax + 1) * (r.umax + 2)) / 2 : 21 + 4 * (r.umax - 5);
    r.nG = r.umax < 6 ? 0 : ((r.umax - 3) * (r.umax - 2)) / 2 - 3;
    r.sS = (r.nS + WAVE - 1) / WAVE;
    r.sG = (r.nG + WAVE - 1) / WAVE;
    r.nit = r.cq ? (sq - 3 + 15) / 16 : 0;                  // qm: 16 lanes per cell
    r.sQ5 = (d - 4 + WAVE - 1) / WAVE;
    r.cqg = (r.cq + 3) / 4;                                 // qm items = groups of 4 cells
    // weights calibrated on per-phase cycle stamps (tools/pf_stamps.py, N = 100,
    // P = 2): ~8 cycles per unit; a closing-pair cell also pays ~210 cycles of
    // chunk set-up, a qm group ~40 + 40 per 16-split step, q5 ~320 per slot
    r.ca = (4 * r.sG + 12 * r.sS) * (P + 1) / 2 + ADX_CA0;
    r.cb = (ADX_CB1 * r.nit + ADX_CB0) * P;
    r.c5 = 40 * r.sQ5 + 40;
    r.Ct = r.c5 + r.cp * r.ca + r.cqg * r.cb;
    return r;
}

// Wave w's items: [qb cells][qm groups][q5] cut into NW equal-cost ranges
// (q5 is last: it belongs to the last wave).  out = kb_lo, kb_hi, km_lo, km_hi.
template <int NW>
__device__ inline void wave_range(const RangeCost &rc, int w, int (&out)[4]) {
    const int lo = w * rc.Ct, hi = lo + rc.Ct;              // x NW
    auto cdiv = [](int x, int y) { return x <= 0 ? 0 : (x + y - 1) / y; };
    out[0] = clampi(cdiv(lo, rc.ca * NW), 0, rc.cp);
    out[1] = clampi(cdiv(hi, rc.ca * NW), 0, rc.cp);
    const int b2 = rc.cp * rc.ca;
    out[2] = 4 * clampi(cdiv(lo - b2 * NW, rc.cb * NW), 0, rc.cqg);
    out[3] = min(rc.cq, 4 * clampi(cdiv(hi - b2 * NW, rc.cb * NW), 0, rc.cqg));
}

// ---------------------------------------------------------------- inside PF
// P variants of one (context, macrostate) folded in lockstep (same cells,
// same pairable set, same factors; the holo variant adds the motif bonus).
// Per-group setup pass (all cells at once, no DP dependency):
//   cc    inner-pair code of every cell,
//   qbm   hairpin (+ ligand motif) factor of every pairable cell,
//   qm1   multiloop-stem factor of every pairable cell, 0 otherwise,
//   pcnt  the number of pairable cells of every diagonal.
// A non-pairable cell keeps qbm = -0.0f for the whole fold (it is never
// finalized, and adds 0 wherever it is read); a wave finds the pairable cells
// of its share of a diagonal by a ballot scan of that sign bit.
// Main loop, ONE barrier per iteration d = 4..N.  Items of iteration d:
//   qb(i, i+d) for the pairable cells   reads qbm spans <= d-2, mla(d-2), qm1(d-1)
//   qm(i, i+d-1) + mla(d-1)             reads qm1 spans <= d-1, qm spans <= d-6
//   q5[d]                               reads qbm spans <= d-1, q5 <= d-1
//   qm1 of the non-pairable cells of d  reads qm1(d-1)
// A closing-pair cell is summed by ONE wave: lanes = terms of its interior-loop
// lists (S and G, dev_types.hpp), reduced with DPP; its multiloop term is the
// split sum mla(i+1, j-1) that the qm item of the previous iteration kept.  A qm
// item is 4 cells x 16 lanes (split points).  Items are cut into NW contiguous
// ranges of equal estimated cost, one per wave.
// Incremental folds.  An MC proposal differs from the walker's current
// sequence at a few positions; a cell (i,j) depends on S[i-1..j+1] only, so
// every cell whose [i-1, j+1] misses the changed positions keeps its value.
// src: the group's tables of the current sequence (HBM, null = fold all);
// dst: where this fold's tables go (null = nowhere); [m_lo, m_hi]: the hull of
// the changed positions, 1-based folded coordinates.  Per diagonal d the
// changed cells are i in [max(1, m_lo-1-d), min(N-d, m_hi+1)]; the qm items
// take one cell more on each side (the multiloop-closing sums of changed
// pairs), q5[j] is recomputed from j = m_lo-1 on.
struct Inc {
    const float *src;
    float *dst;
    int m_lo, m_hi;
    uint8_t *cc_dst;   // MinPlus16: the slot's per-cell codes (dev_types.hpp inc_cc_offset)
};

template <int NT, int P, class SR>
__device__ void pf_group(const KArgs &ka, const int *vs, const uint8_t *raw, const Lds<P> &L,
                         const DevScaled *__restrict__ XS, float (&z)[P], bool &bad, const Inc &inc) {
    constexpr int NW = NT / WAVE;
    const DevVariant V = ka.variants[vs[0]];
    // motif[p]: table p carries a holo variant; NV = 2 packs variants vs[2p], vs[2p+1]
    bool motif[P];
    bool mhalf[2] = {false, false};
#pragma unroll
    for (int p = 0; p < P; p++) {
        motif[p] = false;
        for (int h = 0; h < SR::NV; h++) {
            const bool m = ka.variants[vs[p * SR::NV + h]].motif != 0;
            motif[p] |= m;
            mhalf[h] = m;
        }
    }
    const int N = uni(V.N);
    const float *ct = L.ct;
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);
    const int NP = L.np;
    // incremental fold (Inc): changed cells of diagonal dd are i in [clo, chi],
    // qm items of span s are i in [qlo, qhi]
    const bool incr = inc.src != nullptr;
    const int m_lo = uni(inc.m_lo), m_hi = uni(inc.m_hi);
    auto clo = [&](int dd) { return incr ? max(1, m_lo - 1 - dd) : 1; };
    auto chi = [&](int dd) { return incr ? min(N - dd, m_hi + 1) : N - dd; };
    auto qlo = [&](int sq) { return incr ? max(1, m_lo - 2 - sq) : 1; };
    auto qcount = [&](int sq) {
        if (sq < 4 || sq > N - 3) return 0;
        const int hi = incr ? min(N - sq, m_hi + 2) : N - sq;
        return max(0, hi - qlo(sq) + 1);
    };

    // ---- per-group setup: sequence, constraint arrays, motif sites
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
            const int pp = k - 1;
            if (pp < blen) s = bef[pp];
            else if (pp < blen + ka.Nraw) s = raw[pp - blen];
            else s = aft[pp - blen - ka.Nraw];
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
#pragma unroll
    for (int p = 0; p < P; p++)
        for (int k = tid; k < 2 * NP; k += NT) L.mla[p][k] = SR::zero();
    if constexpr (SR::NV == 2) {   // qm spans N-2, N-1 are never computed: defined for the range guard
        const int C = ((N - 4) * (N - 3)) >> 1;
        for (int k = tid; k < C; k += NT) L.qm[0][k] = SR::zero();
    }
    constrained = __syncthreads_or(constrained);
    if (tid == 0) {
        // ViennaRNA's S1 wrap-around (only reaches values that are never used)
        L.S[0] = L.S[N];
        L.S[N + 1] = L.S[1];
    }
    bool any_motif = false;
#pragma unroll
    for (int p = 0; p < P; p++) any_motif |= motif[p];
    const int mL = XS->motif_len;
    if (any_motif && mL > 0) {
        for (int o = tid + 1; o + mL - 1 <= N; o += NT) {
            bool ok = true;
            for (int k = 0; k < mL && ok; k++) {
                if (L.S[o + k] != XS->motif_code[k]) ok = false;
            }
            for (int k = 0; k < mL && ok; k++) {
                const int pk = XS->motif_pt[k];
                if (pk < 0) ok = L.up[o + k] >= 1;
                else if (pk > k) ok = allowed(L, o + k, o + pk);
            }
            L.mat[o] = ok ? 1 : 0;
        }
    }
    __syncthreads();
    const float sig1 = XS->sig[1];
    const float mlbase_sig = XS->mlbase_sig;
    const float mlclosing = XS->mlclosing;
    const float eTAU = XS->ctab[CT_FSM + 6];
    // packed values: the motif term applies to the holo half only (0x7FFF = no-op for min)
    const float mextra = SR::NV == 2
        ? __uint_as_float((mhalf[0] ? (__float_as_uint(XS->motif_extra) & 0xFFFFu) : 0x7FFFu) |
                          (mhalf[1] ? (__float_as_uint(XS->motif_extra) & 0xFFFF0000u) : 0x7FFF0000u))
        : XS->motif_extra;
    const int nsp = XS->n_special < MAX_SPECIAL_HP ? XS->n_special : MAX_SPECIAL_HP;
    if (tid == 0) {
#pragma unroll
        for (int p = 0; p < P; p++) {
            L.q5[p][0] = SR::one();
            for (int j = 1; j <= 3 && j <= N; j++)
                L.q5[p][j] = (L.up[j] >= 1) ? SR::mul(L.q5[p][j - 1], sig1) : SR::zero();
        }
    }
    // cells of every diagonal: wave w takes diagonals 4 + w, 4 + w + NW, ...
    for (int dd = 4 + wid; dd <= N - 1; dd += NW) {
        const int c = N - dd;
        const int od = off(dd, N);
        const int u = dd - 1;
        int base = 0;
        for (int r0 = 0; r0 < c; r0 += WAVE) {
            const int r = r0 + lane;
            const bool valid = r < c;
            bool pr = false;
            if (valid) {
                const int i = r + 1, j = i + dd;
                const int si = L.S[i], sj = L.S[j], sim = L.S[i - 1], sjp = L.S[j + 1];
                const int type = ptype(si, sj);
                pr = type != 0 && allowed(L, i, j);
                float h = SR::zero(), m1 = SR::zero();
                bool mx = false;
                if (pr) {
                    if (L.up[i + 1] >= u) {
                        bool special = false;
                        if (u == 3 || u == 4 || u == 6) {
                            const uint32_t key = hp_key(L.S, i, u + 2);
                            for (int k = 0; k < nsp; k++)
                                if (XS->sp_key[k] == key) { h = XS->sp_val[k]; special = true; break; }
                        }
                        if (!special)
                            h = SR::mul(L.dt[DT_HP + u],
                                        (u == 3) ? L.dt[DT_TAU + type]
                                                 : L.dt[DT_MMH + type * 25 + L.S[i + 1] * 5 + L.S[j - 1]]);
                    }
                    mx = dd == mL - 1 && mL > 0 && L.mat[i];
                    m1 = L.dt[DT_MLS + type * 25 + sim * 5 + sjp];
                }
#pragma unroll
                for (int p = 0; p < P; p++) {
                    L.qbm[p][od + r] = pr ? ((mx && motif[p]) ? SR::add(h, mextra) : h) : SR::mark();
                    L.qm1[p][colb(j) + i - 1] = m1;
                }
                L.cc[od + r] = static_cast<uint8_t>(rtype(type) * 25 + sjp * 5 + sim);
            }
            base += __popcll(__ballot(pr && r + 1 >= clo(dd) && r + 1 <= chi(dd)));
        }
        if (lane == 0) L.pcnt[dd] = static_cast<uint8_t>(base);   // pairable cells to fold
    }
    __syncthreads();
    const bool has_rec = L.rec || L.rec32;
    if (has_rec) {
        // record offsets: exclusive prefix sum of pcnt over the diagonals (wave 0)
        if (wid == 0) {
            int carry = 0;
            for (int d0 = 0; d0 < N; d0 += WAVE) {
                const int dd = d0 + lane;
                const int own = (dd >= 4 && dd <= N - 1) ? int(L.pcnt[dd]) : 0;
                int v = own;
#pragma unroll
                for (int o = 1; o < WAVE; o <<= 1) {
                    const int t = __shfl_up(v, o, WAVE);
                    if (lane >= o) v += t;
                }
                if (dd <= N) L.rbase[dd] = static_cast<uint16_t>(carry + v - own);
                carry += __shfl(v, WAVE - 1, WAVE);
            }
        }
        __syncthreads();
        // the records, in rank order per diagonal
        for (int dd = 4 + wid; dd <= N - 1; dd += NW) {
            const int c = N - dd, od = off(dd, N), rb = L.rbase[dd];
            int base = 0;
            for (int r0 = 0; r0 < c; r0 += WAVE) {
                const int r = r0 + lane;
                const bool pr = r < c && !SR::is_mark(L.qbm[0][od + r]) && r + 1 >= clo(dd) && r + 1 <= chi(dd);
                const unsigned long long bm = __ballot(pr);
                if (pr) {
                    const int k = rb + base + __popcll(bm & ((1ull << lane) - 1ull));
                    const int i = r + 1, j = i + dd;
                    if (L.rec32) {
                        const int oc = ptype(L.S[i], L.S[j]) * 25 + L.S[i + 1] * 5 + L.S[j - 1];
                        L.rec32[k] = uint32_t(i) | (uint32_t(oc) << 8) | (uint32_t(L.up[i + 1]) << 16) |
                                     (uint32_t(L.dn[j - 1]) << 24);
                    } else {
                        L.rec[k] = static_cast<uint8_t>(i);
                    }
                }
                base += __popcll(bm);
            }
        }
    }
    // item ranges of every (diagonal, wave): rt, or computed in prep() when rt does not fit
    if (L.rt) {
        for (int t = tid; t < (N - 3) * NW; t += NT) {
            const int d = 4 + t / NW, w = t % NW;
            RangeCost rc = range_cost<P>(d, N, d <= N - 1 ? int(L.pcnt[d]) : 0, qcount(d - 1));
            int r[4];
            wave_range<NW>(rc, w, r);
            L.rt[d * NW + w] = uint32_t(r[0]) | (uint32_t(r[1]) << 8) | (uint32_t(r[2]) << 16) | (uint32_t(r[3]) << 24);
        }
    }
    if (L.rt || has_rec) __syncthreads();

    // ---------------- incremental fold: the unchanged cells from the previous tables
    if (incr) {
        const size_t C = size_t(ka.cells);
        for (int dd = 4 + wid; dd <= N - 1; dd += NW) {
            const int lo = clo(dd), hi = chi(dd), od = off(dd, N);
            for (int r = lane; r < N - dd; r += WAVE) {
                const int i = r + 1, j = i + dd;
                if (i >= lo && i <= hi) continue;
#pragma unroll
                for (int p = 0; p < P; p++) {
                    const float *sp = inc.src + p * (3 * C + NP);
                    L.qbm[p][od + r] = sp[od + r];
                    L.qm[p][rowb(i, N) + dd - 4] = sp[C + rowb(i, N) + dd - 4];
                    L.qm1[p][colb(j) + i - 1] = sp[2 * C + colb(j) + i - 1];
                }
            }
        }
        for (int k = tid; k <= m_lo - 2 && k <= N; k += NT) {
#pragma unroll
            for (int p = 0; p < P; p++) L.q5[p][k] = inc.src[p * (3 * C + NP) + 3 * C + k];
        }
        __syncthreads();
    }

    // ---------------- loop-carried state.  prep(d) runs at the end of
    // iteration d-1 (before its barrier) and fills everything iteration d needs
    // that iteration d-1 does not write: item ranges, the first chunk of
    // closing-pair cells, their table prefetch, the term descriptors.
    const DevTables &T = *ka.T;
    int cp = 0, cq = 0, umax = 0, sS = 0, sG = 0, nit = 0, sQ5 = 0;
    int kb_lo = 0, kb_hi = 0, km_lo = 0, km_hi = 0;
    // closing-pair chunk (lanes = cells of the chunk)
    int ci = 1, cty = 0, cA = 0, cB = 0, cidx = 0, cm1 = 0;
    float cmmo = SR::zero(), ctau = SR::one(), cmo = SR::zero(), cm23 = SR::zero(), cmmc = SR::zero();
    float cpm1 = SR::zero(), cmlc = SR::zero(), pfx = SR::zero();
    float cpre[P];
#pragma unroll
    for (int p = 0; p < P; p++) cpre[p] = SR::zero();
    uint8_t *ws = L.wsc + wid * WAVE;
    // term descriptors: offsets advance by k - d per diagonal once every term is
    // valid (d > 36); before that they are recomputed
    TermLanes D;
    int kG[GSLOTS], kS[SSLOTS];
#pragma unroll
    for (int s = 0; s < GSLOTS; s++) {
        const int pk = L.gd[s * WAVE + lane];
        kG[s] = N + 3 + (pk & 255) + (pk >> 8);
    }
#pragma unroll
    for (int s = 0; s < SSLOTS; s++) {
        const int pk = int(L.sd[s * WAVE + lane]);
        const int n1 = pk & 255, n2 = (pk >> 8) & 255, k = pk >> 16;
        kS[s] = N + 3 + n1 + n2;
        D.b1[s] = (k == TK_BUL) ? CT_BUL : (k == TK_1N) ? CT_ONEN : CT_INVMM;
        if (s == 0) {
            D.b2 = (k <= TK_B1) ? CT_STK : (k == TK_M23) ? CT_M23O : CT_ONE;
            D.mwt = (k <= TK_B1) ? -1 : 0;
            D.mwc = (k == TK_M23) ? -1 : 0;
            D.eb = (k == TK_BUL) ? 1.f : 0.f;
            D.em = (k == TK_1N) ? 1.f : 0.f;
            D.e3 = (k == TK_M23) ? 1.f : 0.f;
            D.eg = (k >= TK_I11 && k <= TK_I22) ? 1.f : 0.f;
            D.gsel = (k - TK_I11) & 3;
        } else {
            D.em1 = (k == TK_1N) ? 1.f : 0.f;
        }
    }

    // lanes c < nc: cell kc + c (rank among the pairable cells of diagonal d)
    auto load_chunk = [&](int d, int kc, int nc) {
        const int od = off(d, N);
        uint32_t wc, wp;   // record words of cell `lane` and of cell `lane / 4` of the chunk:
                           //   i | oc << 8 | up[i+1] << 16 | dn[j-1] << 24, oc = type*25 + S[i+1]*5 + S[j-1]
        auto word = [&](int i) {
            const int j = i + d;
            const int oc = ptype(L.S[i], L.S[j]) * 25 + L.S[i + 1] * 5 + L.S[j - 1];
            return uint32_t(i) | (uint32_t(oc) << 8) | (uint32_t(L.up[i + 1]) << 16) | (uint32_t(L.dn[j - 1]) << 24);
        };
        if (L.rec32) {
            const int rb = L.rbase[d] + kc;
            wc = L.rec32[rb + (lane < nc ? lane : nc - 1)];
            wp = L.rec32[rb + ((lane >> 2) < nc ? (lane >> 2) : nc - 1)];
        } else if (L.rec) {
            const int rb = L.rbase[d] + kc;
            wc = word(L.rec[rb + (lane < nc ? lane : nc - 1)]);
            wp = word(L.rec[rb + ((lane >> 2) < nc ? (lane >> 2) : nc - 1)]);
        } else {   // ballot scan of the non-pairable mark -> ws[rank - kc] = i
            int base = 0;
            for (int r0 = 0; r0 < N - d && base < kc + nc; r0 += WAVE) {
                const int r = r0 + lane;
                const bool pr = r < N - d && !SR::is_mark(L.qbm[0][od + r]) && r + 1 >= clo(d) && r + 1 <= chi(d);
                const unsigned long long m = __ballot(pr);
                const int rank = base + __popcll(m & ((1ull << lane) - 1ull));
                if (pr && rank >= kc && rank < kc + nc) ws[rank - kc] = static_cast<uint8_t>(r + 1);
                base += __popcll(m);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            wc = word(ws[lane < nc ? lane : nc - 1]);
            wp = word(ws[(lane >> 2) < nc ? (lane >> 2) : nc - 1]);
        }
        {
            const int i = wc & 255, j = i + d;
            const int oc = (wc >> 8) & 255;
            const int ty = (oc * 41) >> 10, si1 = (oc / 5) % 5, sj1 = oc % 5;
            ci = i;
            cty = ty;
            cA = (wc >> 16) & 255;
            cB = wc >> 24;
            cmmo = L.dt[DT_MMI + oc];
            ctau = ty > 2 ? eTAU : SR::one();
            cmo = SR::mul(ct[CT_ONEN + oc], cmmo);
            cm23 = ct[CT_M23O + oc];
            cidx = od + i - 1;
            cmmc = L.dt[DT_MMI + L.cc[cidx]];
#pragma unroll
            for (int p = 0; p < P; p++) cpre[p] = L.qbm[p][cidx];
            cm1 = colb(j) + i - 1;
            cpm1 = L.qm1[0][cm1];
            cmlc = SR::mul(mlclosing, L.dt[DT_MLS + rtype(ty) * 25 + sj1 * 5 + si1]);
        }
        {   // lane 4c + g: the 1x1 / 1x2 / 2x1 / 2x2 table factor g of cell c (HBM/L2)
            const int c = lane >> 2, g = lane & 3;
            const int n1 = (g >= 2) ? 2 : 1, n2 = (g & 1) ? 2 : 1;
            pfx = SR::zero();
            if (c < nc && n1 + n2 <= umax) {
                const int i = wp & 255, j = i + d;
                const int oc = (wp >> 8) & 255;
                const int typ = (oc * 41) >> 10, a1 = (oc / 5) % 5, b1 = oc % 5;
                const int t2 = (L.cc[off(d - 2 - n1 - n2, N) + i + n1] * 41) >> 10;
                const int sp1 = (n1 == 1) ? a1 : L.S[i + 2], sq1 = (n2 == 1) ? b1 : L.S[j - 2];
                const float *src;
                if (g == 0) src = &T.int11[typ][t2][a1][b1];
                else if (g == 1) src = &T.int21[typ][t2][a1][sq1][b1];
                else if (g == 2) src = &T.int21[t2][typ][sq1][a1][sp1];
                else src = &T.int22[typ][t2][a1][sp1][sq1][b1];
                pfx = *src;
            }
        }
    };

    auto prep = [&](int d) {
        const RangeCost rc = range_cost<P>(d, N, uni((d <= N - 1) ? L.pcnt[d] : 0), qcount(d - 1));
        cp = rc.cp;
        cq = rc.cq;
        umax = rc.umax;
        sS = rc.sS;
        sG = rc.sG;
        nit = rc.nit;
        sQ5 = rc.sQ5;
        const int nS = rc.nS, nG = rc.nG;
        if (L.rt) {
            const uint32_t e = uni(int(L.rt[d * NW + wid]));
            kb_lo = e & 255;
            kb_hi = (e >> 8) & 255;
            km_lo = (e >> 16) & 255;
            km_hi = e >> 24;
        } else {
            int r[4];
            wave_range<NW>(rc, wid, r);
            kb_lo = uni(r[0]);
            kb_hi = uni(r[1]);
            km_lo = uni(r[2]);
            km_hi = uni(r[3]);
        }
        // term descriptors of span d
        if (d <= 36) {
#pragma unroll
            for (int s = 0; s < GSLOTS; s++) {
                const int t = s * WAVE + lane;
                const int u = kG[s] - N - 3, n1 = L.gd[t] & 255;
                const bool ok = t < nG;
                D.offG[s] = ok ? off(d - 2 - u, N) + n1 : 0;
                D.fG[s] = ok ? L.gf[t] : SR::zero();
            }
#pragma unroll
            for (int s = 0; s < SSLOTS; s++) {
                const int t = s * WAVE + lane;
                const int u = kS[s] - N - 3, n1 = int(L.sd[t]) & 255;
                const bool ok = t < nS;
                D.offS[s] = ok ? off(d - 2 - u, N) + n1 : 0;
                D.fS[s] = ok ? L.sf[t] : SR::zero();
            }
        } else {
#pragma unroll
            for (int s = 0; s < GSLOTS; s++) D.offG[s] += kG[s] - d;
#pragma unroll
            for (int s = 0; s < SSLOTS; s++) D.offS[s] += kS[s] - d;
        }
        if (kb_lo < kb_hi) load_chunk(d, kb_lo, (kb_hi - kb_lo) < CHUNK ? kb_hi - kb_lo : CHUNK);
    };

#ifdef ADX_STAMP
    unsigned long long st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
    prep(4);
    for (int d = 4; d <= N; ++d) {
        STAMP(10);
        const int sq = d - 1;
        // ---------------- values iteration d-1 wrote: qm1(i, j-1) and mla(i+1, j-1)
        // of the first chunk; qm1 of the non-pairable cells of d (stored at the end)
        float cprev[P], cml[P];
        auto late = [&]() {
            const int j = ci + d;
            const bool upj = d >= 5 && L.up[j] >= 1;
#pragma unroll
            for (int p = 0; p < P; p++) {
                cprev[p] = upj ? L.qm1[p][colb(j - 1) + ci - 1] : SR::zero();
                cml[p] = SR::mul(L.mla[p][((d - 2) & 1) * NP + ci + 1], cmlc);
            }
        };
        if (kb_lo < kb_hi) late();
        const int r1 = tid, i1 = r1 + 1, j1 = i1 + d;
        const bool has1 = r1 < N - d;
        bool m1np = false;    // non-pairable: the -0 mark (a finalized cell is never -0)
        float m1prev[P];
        int m1up = 0;
        if (has1) {
            m1np = SR::is_mark(L.qbm[0][off(d, N) + i1 - 1]);
#pragma unroll
            for (int p = 0; p < P; p++) m1prev[p] = L.qm1[p][colb(j1 - 1) + i1 - 1];
            m1up = L.up[j1];
        }
        STAMP(0);

        // ---------------- qm(i, i+sq) and mla(i, sq), groups of 4 cells,
        // 16 lanes (split points t = it*16 + l16) per cell:
        // qm[i][jb] = sum_t (pw(t) + qm[i][i+t-1]) * qm1[i+t][jb]
        {
            const int g = lane >> 4, l16 = lane & 15;
            const int tmax = sq - 4;
            const int q0 = qlo(sq);   // first qm cell of this iteration's items
            for (int m0 = km_lo; m0 < km_hi; m0 += 4) {
                const int m = m0 + g;
                const bool cell = m < km_hi;
                const int i = q0 + m, jb = i + sq;
                const int upi = constrained ? L.up[cell ? i : 1] : 255;
                const int o1 = colb(jb) + i - 1, orr = rowb(i, N) - 5;
                float A[P], Pp[P];
#pragma unroll
                for (int p = 0; p < P; p++) { A[p] = SR::zero(); Pp[p] = SR::zero(); }
                for (int it = 0; it < nit; it++) {
                    const int t0 = it * 16 + l16;
                    const bool ok0 = cell && t0 <= tmax;
                    const bool okr = ok0 && t0 >= 5;
                    const float w0 = L.pw[t0 <= N ? t0 : N];
                    const float pw0 = (t0 <= upi) ? w0 : SR::zero();
#pragma unroll
                    for (int p = 0; p < P; p++) {
                        const float v0 = L.qm1[p][o1 + (ok0 ? t0 : 0)];
                        const float r0 = L.qm[p][orr + (okr ? t0 : 5)];
                        const float b0 = ok0 ? v0 : SR::zero();
                        A[p] = SR::fma(okr ? r0 : SR::zero(), b0, A[p]);
                        Pp[p] = SR::fma(pw0, b0, Pp[p]);
                    }
                }
#pragma unroll
                for (int p = 0; p < P; p++) {
                    const float sA = row_sum<SR>(A[p]);
                    const float sP = row_sum<SR>(Pp[p]);
                    if (l16 == 15 && cell) {
                        L.qm[p][rowb(i, N) + sq - 4] = SR::add(sA, sP);
                        L.mla[p][(sq & 1) * NP + i] = sA;
                    }
                }
            }
        }
        STAMP(5);

        // ---------------- qb(i, i+d): lanes = interior-loop terms
        for (int kc = kb_lo; kc < kb_hi; kc += CHUNK) {
            const int nc = (kb_hi - kc) < CHUNK ? kb_hi - kc : CHUNK;
            if (kc != kb_lo) {
                load_chunk(d, kc, nc);
                late();
            }
            float sums[P];
#pragma unroll
            for (int p = 0; p < P; p++) sums[p] = SR::zero();
            // the interior-loop sums of one cell of the chunk (lanes = terms)
            auto cell_terms = [&](int c, float (&part)[P]) {
                CellU u;
                u.i = __builtin_amdgcn_readlane(ci, c);
                u.ty8 = __builtin_amdgcn_readlane(cty, c) * 8;
                u.A = __builtin_amdgcn_readlane(cA, c);
                u.B = __builtin_amdgcn_readlane(cB, c);
                u.mmo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cmmo), c));
                u.tau = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ctau), c));
                u.mo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cmo), c));
                u.m23 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cm23), c));
                const bool masked = constrained && (u.A < umax || u.B < umax);
                // gather of the prefetched 1x1..2x2 table factors for this cell
                const float gtab = __shfl(pfx, c * 4 + D.gsel, WAVE);
                if (masked) qb_terms_dispatch<SR, true, P>(sS, sG, L, D, u, gtab, part);
                else qb_terms_dispatch<SR, false, P>(sS, sG, L, D, u, gtab, part);
            };
            int c = 0;
            if constexpr (P == 1) {
                // two cells per reduction: one permlane32 swap + DPP chain for both,
                // and the two term sweeps are independent (overlapping latencies)
                for (; c + 1 < nc; c += 2) {
                    float pa[1], pb[1], ta, tb;
                    cell_terms(c, pa);
                    cell_terms(c + 1, pb);
                    wave_sum2<SR>(pa[0], pb[0], ta, tb);
                    sums[0] = (lane == c) ? ta : ((lane == c + 1) ? tb : sums[0]);
                }
            }
            for (; c < nc; c++) {
                float part[P], tot[P];
                cell_terms(c, part);
                wave_sums<SR, P>(part, tot);
#pragma unroll
                for (int p = 0; p < P; p++) sums[p] = (lane == c) ? tot[p] : sums[p];
            }
            if (lane < nc) {
#pragma unroll
                for (int p = 0; p < P; p++) {
                    const float qb = SR::add(SR::add(sums[p], cpre[p]), cml[p]);
                    L.qbm[p][cidx] = SR::fin(SR::mul(qb, cmmc));   // never the non-pairable mark
                    L.qm1[p][cm1] = SR::fma(qb, cpm1, SR::mul(cprev[p], mlbase_sig));
                }
            }
        }
        STAMP(4);

        // ---------------- q5[d] (the last wave: q5 is last in the cost order)
        if (wid == NW - 1 && (!incr || d >= m_lo - 1)) {   // q5[j < m_lo - 1] is unchanged
            const int j = d;
            const int sjp = (j < N) ? L.S[j + 1] : 5;
            const int sj = L.S[j];
            float acc[P];
#pragma unroll
            for (int p = 0; p < P; p++) acc[p] = SR::zero();
            for (int q = 0; q < sQ5; q++) {
                const int k0 = q * WAVE + lane + 1;
                const bool ok = k0 <= j - 4;
                const int k = ok ? k0 : 1;
                const int ix = off(j - k, N) + k - 1;
                const int ty = ptype(L.S[k], sj);
                const float e = L.dt[DT_EXT + ty * 36 + ((k > 1) ? L.S[k - 1] : 5) * 6 + sjp];
                const float f = ok ? SR::mul(ct[CT_INVMM + L.cc[ix]], e) : SR::zero();
#pragma unroll
                for (int p = 0; p < P; p++) acc[p] = SR::fma(SR::mul(L.q5[p][k - 1], L.qbm[p][ix]), f, acc[p]);
            }
            float sum[P];
            wave_sums<SR, P>(acc, sum);
            if (lane == 0) {
#pragma unroll
                for (int p = 0; p < P; p++)
                    L.q5[p][j] = SR::add((L.up[j] >= 1) ? SR::mul(L.q5[p][j - 1], sig1) : SR::zero(), sum[p]);
            }
        }
        STAMP(6);
        if (has1 && m1np && i1 >= clo(d) && i1 <= chi(d)) {
#pragma unroll
            for (int p = 0; p < P; p++)
                L.qm1[p][colb(j1) + i1 - 1] = (d >= 5 && m1up >= 1) ? SR::mul(m1prev[p], mlbase_sig) : SR::zero();
        }
        if (d < N) prep(d + 1);
        STAMP(7);
        lds_barrier();   // LDS only: the table prefetch of prep(d+1) stays in flight
        STAMP(9);
    }
#ifdef ADX_STAMP
    if (lane == 0 && wid < 16)
        for (int k = 0; k < 12; k++) atomicAdd(&g_stamps[wid][k], st_acc[k]);
#endif
#pragma unroll
    for (int p = 0; p < P; p++) z[p] = L.q5[p][N];   // scaled Z; energies after the group loop
    if (inc.dst) {   // this fold's tables: the next proposal's unchanged cells
        const size_t C = size_t(ka.cells);
#pragma unroll
        for (int p = 0; p < P; p++) {
            float *dp = inc.dst + p * (3 * C + NP);
            for (int k = tid; k < int(C); k += NT) {
                dp[k] = L.qbm[p][k];
                dp[C + k] = L.qm[p][k];
                dp[2 * C + k] = L.qm1[p][k];
            }
            for (int k = tid; k <= N; k += NT) dp[3 * C + k] = L.q5[p][k];
        }
        if (inc.cc_dst)   // MinPlus16: the codes too (mfe_pair.hip restores them)
            for (int k = tid; k < int(C); k += NT) inc.cc_dst[k] = k < ((N - 4) * (N - 3)) / 2 ? L.cc[k] : 0;
    }
    bad = false;
    if constexpr (SR::NV == 2) {
        // exactness guard of the 16-bit encoding (MinPlus16): every stored value >= floor
        bool low = false;
        const int C = ((N - 4) * (N - 3)) >> 1;
        auto chk = [&](float x) {
            const s16x2 q = MinPlus16::v(x);
            low |= mfe16_inexact(q);
        };
        for (int k = tid; k < C; k += NT) {
            chk(L.qbm[0][k]);
            chk(L.qm[0][k]);
            chk(L.qm1[0][k]);
        }
        for (int k = tid; k <= N; k += NT) chk(L.q5[0][k]);
        bad = __syncthreads_or(low);
    }
}

// ---------------------------------------------------------------- scoring
// lane 0 of the block: score from the per-variant energies in L.G
template <int P>
__device__ double combine_score(const KArgs &ka, const Lds<P> &L, const double *pp, double *terms_out) {
    const DevScaled &X = *ka.X;
    double score = 0.0;
    for (int c = 0; c < ka.n_ctx_eff; c++) {
        for (int t = 0; t < ka.n_terms; t++) {
            const DevTermMap m = ka.tmap[c * ka.n_terms + t];
            double p;
            if (m.kind == 1) {
                // RnaFold::base_pair_prob (scoring.cc:37-51), bppm_kernel; null: the
                // score waits for the outside pass (combine_kernel recomputes it)
                p = pp ? pp[m.pidx] : 0.5;
            } else {
                // vrna_pf returns float (scoring.cc:58,65)
                const double gt = static_cast<double>(static_cast<float>(L.G[m.vfree]));
                const double ga = static_cast<double>(static_cast<float>(L.G[m.vcons]));
                p = exp((gt - ga) / X.kT);
            }
            if (!m.favorable) p = 1.0 - p;
            const double val = log(p);
            if (terms_out) terms_out[c * ka.n_terms + t] = val;
            score += m.weight * val;
        }
    }
    return score;
}

template <int NT, int P, class SR>
__device__ double score_sequence(const KArgs &ka, const DevScaled *__restrict__ XS,
                                 const uint8_t *raw, const Lds<P> &L, const double *pp,
                                 float *dG_out, double *terms_out, bool &any_bad, int w) {
    const int ng = P * SR::NV == 2 ? ka.n_groups2 : ka.n_variants;
    any_bad = false;
    for (int g = 0; g < ng; g++) {
        int vs[P * SR::NV];
        if constexpr (P * SR::NV == 2) {
            vs[0] = ka.groups2[2 * g];
            vs[1] = ka.groups2[2 * g + 1];
        } else {
            vs[0] = g;
        }
        float z[P];
        bool bad = false;
        Inc inc{nullptr, nullptr, 0, 0, nullptr};
        if (ka.tab) {   // MC state: read the current tables, write this proposal's
            const size_t G = inc_group_floats(ka.cells, ka.Nmax, P);
            const int cur = ka.cur_slot[w];
            float *base = ka.tab + size_t(w) * 2 * ka.tab_slot;
            inc.dst = base + size_t(1 - cur) * ka.tab_slot + size_t(g) * G;
            if constexpr (P == 1 && SR::NV == 2)
                inc.cc_dst = reinterpret_cast<uint8_t *>(base + size_t(1 - cur) * ka.tab_slot +
                                                         inc_cc_offset(ka.cells, ka.Nmax, ka.n_groups2, g));
            if constexpr (P == 2 && SR::NV == 1 && !SR::MFE)   // PF groups (pf_cells.hip restores the codes)
                inc.cc_dst = reinterpret_cast<uint8_t *>(base + size_t(1 - cur) * ka.tab_slot +
                                                         inc_cc_offset_pf(ka.cells, ka.Nmax, ka.n_groups2, g));
            if (ka.tab_valid[w] && ka.chg && ka.chg[2 * w] >= 0) {
                const int lb = ka.variants[vs[0]].before_len;
                inc.src = base + size_t(cur) * ka.tab_slot + size_t(g) * G;
                inc.m_lo = ka.chg[2 * w] + 1 + lb;
                inc.m_hi = ka.chg[2 * w + 1] + 1 + lb;
            }
        }
        pf_group<NT, P, SR>(ka, vs, raw, L, XS, z, bad, inc);
        any_bad |= bad;
        if (threadIdx.x == 0) {
            if constexpr (SR::NV == 2) {
                const s16x2 q = MinPlus16::v(z[0]);
                L.G[vs[0]] = (q.x >= 0x4000) ? double(MFE_BIG) : static_cast<double>(q.x);
                L.G[vs[1]] = (q.y >= 0x4000) ? double(MFE_BIG) : static_cast<double>(q.y);
            } else {
#pragma unroll
                for (int p = 0; p < P; p++) L.G[vs[p]] = static_cast<double>(z[p]);
            }
        }
        __syncthreads();   // the next group rewrites the tables
    }
    double s = 0.0;
    if (threadIdx.x == 0) {
        for (int v = 0; v < ka.n_variants; v++) {
            const int N = ka.variants[v].N;
            double g;
            if constexpr (SR::MFE)   // f5[N] in dcal/mol; BIG and above = no structure
                g = (L.G[v] >= 0.5 * double(MFE_BIG)) ? double(INFINITY) : L.G[v] / 100.0;
            else                     // ensemble energy -kT (ln Z_scaled - N ln sigma), as vrna_pf (float)
                g = -XS->kT * (log(L.G[v]) - N * XS->log_sigma);
            L.G[v] = g;
            if (dG_out) dG_out[v] = static_cast<float>(g);
        }
        s = combine_score(ka, L, pp, terms_out);
    }
    return s;
}

// combine_score's arithmetic (scoring.cc:53-71): term idx (= context * n_terms
// + term) of the walker whose per-variant energies are g and pair
// probabilities pp (null: the pair terms read 0.5)
__device__ __forceinline__ double term_value(const KArgs &ka, const float *g, const double *pp, int idx,
                                             double &weight) {
    const DevTermMap m = ka.tmap[idx];
    double p = (m.kind == 1) ? (pp ? pp[m.pidx] : 0.5)
                             : exp((static_cast<double>(g[m.vfree]) - static_cast<double>(g[m.vcons])) / ka.X->kT);
    if (!m.favorable) p = 1.0 - p;
    weight = m.weight;
    return log(p);
}

// The score of walker w from KArgs::gstep, one wave: the terms' values on
// lanes, summed in term order (the same sum as combine_kernel's loop); tv
// (the walker's term values, optional).  Result uniform.
__device__ double combine_wave(const KArgs &ka, int w, int lane, double *tv) {
    const float *g = ka.gstep + size_t(w) * ka.n_variants;
    const double *pp = ka.pair_p ? ka.pair_p + size_t(w) * ka.n_pairs : nullptr;
    const int nt = ka.n_terms * ka.n_ctx_eff;
    double score = 0.0;
    for (int b0 = 0; b0 < nt; b0 += WAVE) {
        const int idx = b0 + lane;
        double val = 0.0, wt = 0.0;
        if (idx < nt) {
            val = term_value(ka, g, pp, idx, wt);
            if (tv) tv[idx] = val;
        }
        const int n = min(WAVE, nt - b0);
        for (int k = 0; k < n; k++) score += __shfl(wt, k, WAVE) * __shfl(val, k, WAVE);
    }
    return score;
}

template <int NT, int P, class SR>
__global__ void __launch_bounds__(NT, (NT >= 1024) ? 4 : (NT > 512) ? 3 : (P == 2 ? 2 : 4))   // min waves per SIMD
score_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, double *scores,
             double *terms, float *dG, const int *mask) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Lds<P> L;
    lds_layout<false, P>(smem, ka.cells, ka.Nmax, ka.n_variants, &L, ka.opt & 3, (ka.opt & 4) != 0, NT / WAVE);
    auto fold_one = [&](int w) {
        load_ctab(ka, L);
        for (int k = threadIdx.x; k < ka.Nraw; k += NT) L.raw[k] = seqs[size_t(w) * ka.Nraw + k];
        __syncthreads();
        const int nt = ka.n_terms * ka.n_ctx_eff;
        const double *pp = ka.pair_p ? ka.pair_p + size_t(w) * ka.n_pairs : nullptr;
        bool bad = false;
        const double s = score_sequence<NT, P, SR>(ka, XS, L.raw, L, pp, dG ? dG + size_t(w) * ka.n_variants : nullptr,
                                              terms ? terms + size_t(w) * nt : nullptr, bad, w);
        if (threadIdx.x == 0) {
            scores[w] = s;
            if (SR::NV == 2 && bad && ka.ovf) {
                ka.ovf[w] = 1;                         // re-folded by the FP32 MinPlus kernel
                if (ka.tab) ka.tab_valid[w] = 0;       // and folded from scratch next time
            }
        }
        __syncthreads();   // the LDS tables are the next walker's
    };
    if (int(gridDim.x) >= W) {   // one walker per workgroup
        const int w = blockIdx.x;
        if (SR::NV == 2 && ka.ovf && threadIdx.x == 0) ka.ovf[w] = 0;
        if (mask && mask[w] != 1) return;  // MC: only walkers whose proposal changed
        fold_one(w);
        return;
    }
    // a short grid (the FP32 refold of the few walkers whose 16-bit fold left the
    // exact range, launch_score_m): each workgroup scans its contiguous share of
    // the mask 64 flags per load (every wave takes the same ballot) and folds
    // the flagged walkers
    const int per = (W + int(gridDim.x) - 1) / int(gridDim.x);
    const int lo = int(blockIdx.x) * per, hi = min(W, lo + per);
    const int lane = threadIdx.x & (WAVE - 1);
    for (int base = lo; base < hi; base += WAVE) {
        const int wl = base + lane;
        uint64_t m = __ballot(wl < hi && (!mask || mask[wl] == 1));
        while (m) {
            const int q = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            fold_one(base + q);
        }
    }
}

// ---------------------------------------------------------------- outside / bppm
// Base-pair probabilities of one fold (ViennaRnaFold::base_pair_prob,
// scoring.cc:37-51; vrna_pf with compute_bpp): P(i,j) = qb(i,j) * qbb(i,j) / Z,
// qbb = dZ/dqb the outside (adjoint) quantity of the inside recursions of
// pf_group, in gather form and descending span (oracle/fold.c orc_bppm is the
// scatter form of the same sweep):
//   q5b[m]   = [up[m+1]] sigma q5b[m+1] + sum_j q5b[j] qb(m+1,j) ext(m+1,j)
//   qmb(i,j) = sum_{l>j} Y(i,l) qm1(j+1,l),  Y(i,l) = qmb(i,l) + X(i,l),
//              X(i,l) = qbb(i-1,l+1) MLclosing stemM(rev(i-1,l+1))
//   qm1b(k,l)= qmb(k,l) + sum_{i<k} [qmb(i,l) pw(k-i) + Y(i,l) qm(i,k-1)]
//              + [up[l+1]] expMLbase sigma qm1b(k,l+1)
//   qbb(p,q) = q5b[q] q5[p-1] ext(p,q) + qm1b(p,q) stemM(p,q)
//              + sum_{(i,j) enclosing, loop <= 30} qbb(i,j) F_interior(i,j,p,q)
// One wave per cell (lanes = split points / interior-loop terms), one barrier
// per diagonal.  The interior gather mirrors qb_terms: qbb is stored times the
// outer pair's mismatch, special loops cancel it with the same CT_* tables
// indexed by the outer pair's code.
struct Outs {
    float *qbb;    // diagonal-major: qbb(i,j) * mismatchI(outer code), 0 for non-pairable cells
    float *qmb;    // column-major colb(j)+i-1
    float *Y;      // row-major rowb(i)+j-i-4
    float *qm1b;   // [2][NP] the last two diagonals, by i
    float *q5b;    // [NP]
    float *pm;     // [NP] motif site weights qbb(o, o+L-1) * extra / Z, by site start
};

// LDS carve of the outside arrays after the inside layout.  GOUT: the three
// cell tables (qbb, qmb, Y) live in a per-workgroup global scratch slice
// instead (devices whose inside + outside tables exceed one CU's LDS, e.g.
// N = 150); the rest stays in LDS.  (A column-major copy of Y for coalesced
// r2 reads was measured slower: 58.4 vs 53.7 ms at N = 150.)
template <bool DRY, bool GOUT>
__host__ __device__ inline size_t outs_layout(char *base, size_t o, int cells, int Nmax, Outs *O,
                                              char *gbase = nullptr) {
    auto take = [&](size_t bytes) -> char * {
        char *p = DRY ? nullptr : base + o;
        o += (bytes + 15) & ~size_t(15);
        return p;
    };
    size_t g = 0;
    auto gtake = [&](size_t bytes) -> char * {
        char *p = DRY ? nullptr : gbase + g;
        g += (bytes + 15) & ~size_t(15);
        return p;
    };
    const size_t C = size_t(cells);
    const int NP = Nmax + 2;
    Outs t;
    t.qbb = reinterpret_cast<float *>(GOUT ? gtake(C * 4) : take(C * 4));
    t.qmb = reinterpret_cast<float *>(GOUT ? gtake(C * 4) : take(C * 4));
    t.Y = reinterpret_cast<float *>(GOUT ? gtake(C * 4) : take(C * 4));
    t.qm1b = reinterpret_cast<float *>(take(2 * NP * 4));
    t.q5b = reinterpret_cast<float *>(take(NP * 4));
    t.pm = reinterpret_cast<float *>(take(NP * 4));
    if (!DRY) *O = t;
    return o;
}
// global scratch bytes per workgroup of the GOUT layout
__host__ __device__ inline size_t outs_global_bytes(int cells) {
    return 3 * ((size_t(cells) * 4 + 15) & ~size_t(15));
}

// full: row stride ld (folded coordinates, 0-based), pre-zeroed by the host;
// pp: the requested pairs of this variant (KArgs::pairs with bvars index bv).
template <int NT>
__device__ void outside(const KArgs &ka, int v, int bv, const Lds<1> &L, const Outs &O,
                        const DevScaled *__restrict__ XS, float Z, double *full, int ld, double *pp) {
    constexpr int NW = NT / WAVE;
    const DevVariant V = ka.variants[v];
    const int N = uni(V.N);
    const int tid = threadIdx.x;
    const int lane = tid & (WAVE - 1);
    const int wid = uni(tid / WAVE);
    const int NP = L.np;
    const float *ct = L.ct;
    const uint8_t *S = L.S;
    const float sig1 = XS->sig[1];
    const float mlbase_sig = XS->mlbase_sig;
    const float mlclosing = XS->mlclosing;
    const float eTAU = XS->ctab[CT_FSM + 6];
    const bool motif = V.motif != 0 && XS->motif_len > 0;
    const int mL = XS->motif_len;
    const DevTables &T = *ka.T;
    // outer code of pair (a, b): type * 25 + S[a+1] * 5 + S[b-1]
    auto ocode = [&](int a, int b) { return ptype(S[a], S[b]) * 25 + S[a + 1] * 5 + S[b - 1]; };

    // ---- setup: zeroed adjoints
    for (int dd = 4 + wid; dd <= N - 1; dd += NW) {
        const int od = off(dd, N);
        for (int r = lane; r < N - dd; r += WAVE) {
            const int i = r + 1, j = i + dd;
            O.qbb[od + r] = 0.f;
            O.qmb[colb(j) + i - 1] = 0.f;
            O.Y[rowb(i, N) + dd - 4] = 0.f;
        }
    }
    for (int k = tid; k < 2 * NP; k += NT) O.qm1b[k] = 0.f;
    for (int k = tid; k < NP; k += NT) { O.q5b[k] = 0.f; O.pm[k] = 0.f; }
    __syncthreads();

    // ---- exterior adjoint q5b (one wave, sequential in m)
    if (wid == 0) {
        if (lane == 0) O.q5b[N] = 1.f;
        float nxt = 1.f;   // q5b[m + 1]
        for (int m = N - 1; m >= 0; m--) {
            const int k = m + 1;
            float acc = 0.f;
            for (int j = k + 4 + lane; j <= N; j += WAVE) {
                const int ix = off(j - k, N) + k - 1;
                const int ty = ptype(S[k], S[j]);
                const float e = L.dt[DT_EXT + ty * 36 + ((k > 1) ? S[k - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
                acc = fmaf(O.q5b[j] * L.qbm[0][ix], ct[CT_INVMM + L.cc[ix]] * e, acc);
            }
            const float val = ((L.up[k] >= 1) ? nxt * sig1 : 0.f) + wave_sum(acc);
            if (lane == 0) O.q5b[m] = val;
            nxt = val;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();

    // ---- per-lane term descriptors (S list: 2 slots, G list: 6 slots)
    int sn1[SSLOTS], sn2[SSLOTS], skd[SSLOTS];
    float sfv[SSLOTS];
#pragma unroll
    for (int s = 0; s < SSLOTS; s++) {
        const int pk = int(L.sd[s * WAVE + lane]);
        sn1[s] = pk & 255;
        sn2[s] = (pk >> 8) & 255;
        skd[s] = (s * WAVE + lane < XS->s_cnt[31]) ? (pk >> 16) : -1;
        sfv[s] = L.sf[s * WAVE + lane];
    }
    int gn1[GSLOTS], gu[GSLOTS];
    float gfv[GSLOTS];
#pragma unroll
    for (int s = 0; s < GSLOTS; s++) {
        const int pk = L.gd[s * WAVE + lane];
        gn1[s] = pk & 255;
        gu[s] = (s * WAVE + lane < XS->g_cnt[31]) ? gn1[s] + (pk >> 8) : 99;
        gfv[s] = L.gf[s * WAVE + lane];
    }

    for (int d = N - 1; d >= 4; d--) {
        const int nc = N - d;
        const int od = off(d, N);
        const int umax = min(MAXLOOP_K, N - 3 - d);
        // cells r = wid + k*NW of this wave: lane k keeps cell k's three sums and
        // finishes it in the parallel tail below
        float v_qmb = 0.f, v_rest = 0.f, v_int = 0.f;
        // Y(i, j) of the lane's tail cell (X(i, j), stored two diagonals ago; no
        // wave writes span d before the tail), read now so the tail's update is a store
        float y_old;
        {
            const int kc = (nc - wid + NW - 1) / NW;
            const int i = lane < kc ? wid + lane * NW + 1 : 1;
            y_old = O.Y[lane < kc ? rowb(i, N) + d - 4 : 0];
        }
        int k = 0;
        for (int r = wid; r < nc; r += NW, k++) {
            const int i = r + 1, j = i + d;
            const int idx = od + r;
            const bool pr = !SumProd::is_mark(L.qbm[0][idx]);
            // multiloop adjoints: split points over lanes.  Every read below is
            // unconditional (a masked lane reads a valid cell and discards it by a
            // select): a read under a per-lane branch waits for memory before the
            // next one issues, and with the outside tables in global scratch
            // (GOUT) each wait is a global-memory round trip.
            float a_qmb = 0.f, a_rest = 0.f;
            struct MlQ { float y[2], q[2]; bool ok[2]; };
            struct MlR { float qv[2], yv[2], mv[2], pv[2]; int t[2]; bool ok[2], up[2]; };
            auto q_load = [&](int l0, MlQ &m) {   // qmb split points l0 + lane, l0 + 64 + lane
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int l = l0 + h * WAVE + lane;
                    m.ok[h] = l <= N;
                    m.y[h] = O.Y[m.ok[h] ? rowb(i, N) + l - i - 4 : 0];
                    m.q[h] = L.qm1[0][m.ok[h] ? colb(l) + j : 0];
                }
            };
            auto q_acc = [&](const MlQ &m) {
#pragma unroll
                for (int h = 0; h < 2; h++) a_qmb = m.ok[h] ? fmaf(m.y[h], m.q[h], a_qmb) : a_qmb;
            };
            auto r_load = [&](int p0, MlR &m) {   // r2 / qmb-chain split points p0 + lane, p0 + 64 + lane
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int ip = p0 + h * WAVE + lane;
                    m.ok[h] = ip < i;
                    m.t[h] = i - ip;
                    const int ips = m.ok[h] ? ip : 1, ts = m.ok[h] ? m.t[h] : 0;
                    const bool l5 = m.ok[h] && m.t[h] >= 5;
                    m.qv[h] = O.qmb[colb(j) + ips - 1];
                    m.pv[h] = L.pw[ts];
                    m.up[h] = L.up[ips] >= ts;
                    m.yv[h] = O.Y[l5 ? rowb(ip, N) + j - ip - 4 : 0];
                    m.mv[h] = L.qm[0][l5 ? rowb(ip, N) + m.t[h] - 5 : 0];
                }
            };
            auto r_acc = [&](const MlR &m) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    float x = m.up[h] ? m.qv[h] * m.pv[h] : 0.f;
                    x = m.t[h] >= 5 ? fmaf(m.yv[h], m.mv[h], x) : x;
                    a_rest = m.ok[h] ? a_rest + x : a_rest;
                }
            };
            // the first 128 split points of both sums are read before the interior
            // loops and summed after them (one batch of reads per cell at N <= 133)
            MlQ mq;
            MlR mr;
            q_load(j + 5, mq);
            r_load(1, mr);
            // interior loops (p, q) = (i, j) inside (a, b) = (i-1-n1, j+1+n2)
            float a_int = 0.f;
            if (pr) {
                const int ccode = L.cc[idx];
                const int ty2 = (ccode * 41) >> 10;
                const float mmin = L.dt[DT_MMI + ccode];
                const float tau_in = ty2 > 2 ? eTAU : 1.f;
                const float mo_in = ct[CT_ONEN + ccode] * mmin;
                const float m23_in = ct[CT_M23O + ccode];
                const int A = min(int(L.dn[i - 1]), i - 2), B = min(int(L.up[j + 1]), N - 1 - j);
                float gv[GSLOTS];
                bool gok[GSLOTS];
#pragma unroll
                for (int s = 0; s < GSLOTS; s++) {
                    const int n1 = gn1[s], u = gu[s], n2 = u - n1;
                    gok[s] = u <= umax && n1 <= A && n2 <= B;
                    gv[s] = O.qbb[gok[s] ? off(d + 2 + u, N) + i - 2 - n1 : idx];
                }
                float sv[SSLOTS], stv[SSLOTS], sf[SSLOTS];
                bool sok[SSLOTS], stab[SSLOTS];
#pragma unroll
                for (int s = 0; s < SSLOTS; s++) {
                    const int n1 = sn1[s], n2 = sn2[s], k = skd[s], u = n1 + n2;
                    sok[s] = k >= 0 && u <= umax && n1 <= A && n2 <= B;
                    const int a = sok[s] ? i - 1 - n1 : i, b = sok[s] ? j + 1 + n2 : j;   // masked: the cell itself
                    sv[s] = O.qbb[sok[s] ? off(d + 2 + u, N) + a - 1 : idx];
                    const int ocd = ocode(a, b);   // from S (no dependent scratch load)
                    const int t1 = (ocd * 41) >> 10;
                    // select form of the qb_terms factors (no divergent branches):
                    // base (outer code) x second table factor x uniform inner factor
                    const int base = (k == TK_BUL) ? CT_BUL : (k == TK_1N) ? CT_ONEN : CT_INVMM;
                    const int sec = (k <= TK_B1) ? CT_STK + t1 * 8 + ty2 : (k == TK_M23) ? CT_M23O + ocd : CT_ONE;
                    const float um = (k == TK_BUL) ? tau_in : (k == TK_1N) ? mo_in : (k == TK_M23) ? m23_in : 1.f;
                    // 1x1, 1x2, 2x1, 2x2 tables (HBM / L2): the address selected, the load unconditional
                    const int a1 = S[a + 1], b1 = S[b - 1], sp1 = S[i - 1], sq1 = S[j + 1];
                    const float *src = (k == TK_I11) ? &T.int11[t1][ty2][a1][b1]
                                     : (k == TK_I12) ? &T.int21[t1][ty2][a1][sq1][b1]
                                     : (k == TK_I21) ? &T.int21[ty2][t1][sq1][a1][sp1]
                                     : &T.int22[t1][ty2][a1][sp1][sq1][b1];
                    stab[s] = k >= TK_I11 && k <= TK_I22;
                    stv[s] = *src;
                    sf[s] = ct[base + ocd] * ct[sec] * um;
                }
                float g = 0.f;
#pragma unroll
                for (int s = 0; s < GSLOTS; s++) g = gok[s] ? fmaf(gv[s], gfv[s], g) : g;
                float sp = 0.f;
#pragma unroll
                for (int s = 0; s < SSLOTS; s++)
                    sp = sok[s] ? fmaf(sv[s], sf[s] * ((stab[s] ? stv[s] : 1.f) * sfv[s]), sp) : sp;
                a_int = fmaf(g, mmin, sp);
            }
            q_acc(mq);
            for (int l0 = j + 5 + 2 * WAVE; l0 <= N; l0 += 2 * WAVE) {
                q_load(l0, mq);
                q_acc(mq);
            }
            r_acc(mr);
            for (int p0 = 1 + 2 * WAVE; p0 < i; p0 += 2 * WAVE) {
                r_load(p0, mr);
                r_acc(mr);
            }
            float s_qmb, s_rest;
            wave_sum2<SumProd>(a_qmb, a_rest, s_qmb, s_rest);
            const float s_int = wave_sum(a_int);
            v_qmb = (lane == k) ? s_qmb : v_qmb;
            v_rest = (lane == k) ? s_rest : v_rest;
            v_int = (lane == k) ? s_int : v_int;
        }
        if (lane < k) {
            const int r = wid + lane * NW;
            const int i = r + 1, j = i + d;
            const int idx = od + r;
            const bool pr = !SumProd::is_mark(L.qbm[0][idx]);
            const float chain = (j < N && L.up[j + 1] >= 1) ? mlbase_sig * O.qm1b[((d + 1) & 1) * NP + i] : 0.f;
            const float qm1b_v = v_qmb + v_rest + chain;
            O.qmb[colb(j) + i - 1] = v_qmb;
            O.Y[rowb(i, N) + d - 4] = y_old + v_qmb;   // X(i, j) + qmb(i, j)
            O.qm1b[(d & 1) * NP + i] = qm1b_v;
            float qbbm = 0.f;
            if (pr) {
                const int ty = ptype(S[i], S[j]);
                const float ext = L.dt[DT_EXT + ty * 36 + ((i > 1) ? S[i - 1] : 5) * 6 + ((j < N) ? S[j + 1] : 5)];
                const float stem = L.dt[DT_MLS + ty * 25 + S[i - 1] * 5 + S[j + 1]];
                const float qbb_v = v_int + O.q5b[j] * L.q5[0][i - 1] * ext + qm1b_v * stem;
                qbbm = qbb_v * L.dt[DT_MMI + ocode(i, j)];
                if (d - 2 >= 4)   // X(i+1, j-1): this pair closing a multiloop
                    O.Y[rowb(i + 1, N) + d - 6] =
                        qbb_v * mlclosing * L.dt[DT_MLS + rtype(ty) * 25 + S[j - 1] * 5 + S[i + 1]];
                const double qb = double(L.qbm[0][idx]) * double(ct[CT_INVMM + L.cc[idx]]);
                if (full) {
                    const double pij = qb * double(qbb_v) / double(Z);
                    full[size_t(i - 1) * ld + (j - 1)] = pij;
                    full[size_t(j - 1) * ld + (i - 1)] = pij;
                }
                if (motif && d == mL - 1 && L.mat[i]) O.pm[i] = float(double(qbb_v) * XS->motif_extra / Z);
            }
            O.qbb[idx] = qbbm;
        }
        __syncthreads();
    }
    // ---- the motif's inner pairs (the extra term at its closing cell)
    if (motif && full && tid == 0) {
        for (int o = 1; o + mL - 1 <= N; o++) {
            if (O.pm[o] == 0.f) continue;
            for (int k = 1; k < mL - 1; k++) {
                const int pk = XS->motif_pt[k];
                if (pk > k) {
                    full[size_t(o + k - 1) * ld + (o + pk - 1)] += O.pm[o];
                    full[size_t(o + pk - 1) * ld + (o + k - 1)] += O.pm[o];
                }
            }
        }
    }
    // ---- requested pairs of this variant (score terms)
    if (pp) {
        for (int t = tid; t < ka.n_pairs; t += NT) {
            if (ka.pairs[3 * t] != bv) continue;
            const int i = ka.pairs[3 * t + 1], j = ka.pairs[3 * t + 2];
            double pij = 0.0;
            if (i >= 1 && j <= N && j - i >= 4) {
                const int idx = off(j - i, N) + i - 1;
                if (!SumProd::is_mark(L.qbm[0][idx])) {
                    const double qb = double(L.qbm[0][idx]) * double(ct[CT_INVMM + L.cc[idx]]);
                    const double qbb = double(O.qbb[idx]) / double(L.dt[DT_MMI + ocode(i, j)]);
                    pij = qb * qbb / double(Z);
                }
                if (motif)
                    for (int o = 1; o + mL - 1 <= N; o++) {
                        if (O.pm[o] == 0.f || i < o || j > o + mL - 1) continue;
                        const int pk = XS->motif_pt[i - o];
                        if (i - o >= 1 && pk == j - o) pij += O.pm[o];
                    }
            }
            pp[t] = pij;
        }
    }
}

// One workgroup per (walker, outside variant): inside (pf_group, P = 1) then
// outside.  full: [W][n_bvars][ld*ld] or null; pair_p: [W][n_pairs] or null;
// GOUT: gscratch holds gridDim.x slices of outs_global_bytes.
// reuse: the proposal's inside tables were just written by score_kernel to the
// walker's next slot (KArgs::tab, score P = sp): pf_group restores every cell
// from there (an incremental fold with nothing changed) instead of refolding.
template <int NT, bool GOUT>
__global__ void __launch_bounds__(NT, 1)
bppm_kernel(KArgs ka, const DevScaled *__restrict__ XS, const uint8_t *seqs, int W, const int *mask,
            double *full, int ld, double *pair_p, char *gscratch, int sp, int reuse) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Lds<1> L;
    const size_t o = lds_layout<false, 1>(smem, ka.cells, ka.Nmax, ka.n_variants, &L, 0, false);
    Outs O;
    outs_layout<false, GOUT>(smem, o, ka.cells, ka.Nmax, &O,
                             GOUT ? gscratch + size_t(blockIdx.x) * outs_global_bytes(ka.cells) : nullptr);
    const int w = blockIdx.x / ka.n_bvars, bv = blockIdx.x % ka.n_bvars;
    if (w >= W) return;
    if (mask && mask[w] != 1) return;
    load_ctab(ka, L);
    for (int k = threadIdx.x; k < ka.Nraw; k += NT) L.raw[k] = seqs[size_t(w) * ka.Nraw + k];
    __syncthreads();
    const int v = ka.bvars[bv];
    const int vs[1] = {v};
    float z[1];
    bool bad = false;
    Inc inc{nullptr, nullptr, 0, 0, nullptr};
    if (reuse && ka.tab) {
        const size_t B = 3 * size_t(ka.cells) + size_t(ka.Nmax) + 2;   // one variant's tables
        // score P = 1: group = variant; P = 2: the groups2 position (host-computed)
        const size_t o = (sp == 2 ? size_t(ka.bvar_slot[bv]) : size_t(v)) * B;
        const int cur = ka.cur_slot[w];
        inc.src = ka.tab + size_t(w) * 2 * ka.tab_slot + size_t(1 - cur) * ka.tab_slot + o;
        inc.m_lo = 4 * ka.Nmax + 8;   // no changed cell: every cell and q5 from src
        inc.m_hi = -8;
    }
    pf_group<NT, 1, SumProd>(ka, vs, L.raw, L, XS, z, bad, inc);
    __syncthreads();
    outside<NT>(ka, v, bv, L, O, XS, z[0],
                full ? full + (size_t(w) * ka.n_bvars + bv) * size_t(ld) * ld : nullptr, ld,
                pair_p ? pair_p + size_t(w) * ka.n_pairs : nullptr);
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

// Orders a wave's LDS accesses around it (the LDS executes one wave's
// instructions in order; this keeps the compiler from moving them across):
// the MC step's waves each own their LDS and never wait for one another.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A walker's MT19937 stream (MT_WORDS words in HBM: state + index) as a step
// reads it: only the words [lo, hi) it will draw are staged in LDS (a step
// draws a few), the whole state only when it twists (then written back).
struct MtView {
    uint32_t *mt;          // LDS, words [lo, hi) valid
    const uint32_t *g;     // HBM state
    int idx, lo, hi;
    bool twisted;
};

__device__ uint32_t mt_next(MtView &g, int lane) {
    if (g.idx >= 624) {
        if (g.lo != 0 || g.hi != 624) {
            for (int k = lane; k < 624; k += WAVE) g.mt[k] = g.g[k];
            wave_sync();
            g.lo = 0;
            g.hi = 624;
        }
        mt_twist_wave(g.mt, lane);
        g.idx = 0;
        g.twisted = true;
    }
    uint32_t y = (g.idx < g.hi) ? g.mt[g.idx] : g.g[g.idx];   // past the window: a rejection draw
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

// ---------------------------------------------------------------- median
// std::nth_element(a, a + k, a + n) over doubles with operator<, following
// libstdc++ 11's introselect (<bits/stl_algo.h> __introselect,
// __unguarded_partition_pivot, __move_median_to_first, __insertion_sort;
// <bits/stl_heap.h> __heap_select / __adjust_heap / __push_heap) compare for
// compare and swap for swap.  AutoScalingThermostat::adjust calls it on its
// training set (sampling.cc:389-393); keeping the same order of operations
// puts the same element at k even among +0.0 / -0.0 ties and NaNs.  Run by one
// lane on the walker's training buffer (<= period doubles, once per period).
__device__ __forceinline__ void nth_swap(double *a, int i, int j) {
    const double t = a[i];
    a[i] = a[j];
    a[j] = t;
}

__device__ void nth_adjust_heap(double *a, int hole, int len, double v) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (a[child] < a[child - 1]) child--;
        a[hole] = a[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        a[hole] = a[child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && a[parent] < v) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = v;
}

__device__ void nth_element_libstdcxx(double *a, int k, int n) {
    if (n == 0 || k == n) return;
    int first = 0, last = n;
    int depth = 2 * (31 - __clz(n));
    while (last - first > 3) {
        if (depth == 0) {
            // __heap_select(first, k + 1, last) then iter_swap(first, k)
            double *h = a + first;
            const int mid = k + 1 - first, len = last - first;
            if (mid >= 2)
                for (int p = (mid - 2) / 2;; p--) {
                    nth_adjust_heap(h, p, mid, h[p]);
                    if (p == 0) break;
                }
            for (int i = mid; i < len; i++)
                if (h[i] < h[0]) {
                    const double v = h[i];
                    h[i] = h[0];
                    nth_adjust_heap(h, 0, mid, v);
                }
            nth_swap(a, first, k);
            return;
        }
        --depth;
        // __unguarded_partition_pivot: median of (first+1, mid, last-1) to first
        const int m = first + (last - first) / 2, x = first + 1, z = last - 1;
        int pick;
        if (a[x] < a[m]) pick = (a[m] < a[z]) ? m : (a[x] < a[z]) ? z : x;
        else pick = (a[x] < a[z]) ? x : (a[m] < a[z]) ? z : m;
        nth_swap(a, first, pick);
        int lo = first + 1, hi = last;
        for (;;) {
            while (a[lo] < a[first]) lo++;
            hi--;
            while (a[first] < a[hi]) hi--;
            if (!(lo < hi)) break;
            nth_swap(a, lo, hi);
            lo++;
        }
        if (lo <= k) first = lo;
        else last = lo;
    }
    // __insertion_sort(first, last)
    for (int i = first + 1; i < last; i++) {
        const double v = a[i];
        if (v < a[first]) {
            for (int j = i; j > first; j--) a[j] = a[j - 1];
            a[first] = v;
        } else {
            int hole = i;
            while (v < a[hole - 1]) {
                a[hole] = a[hole - 1];
                hole--;
            }
            a[hole] = v;
        }
    }
}

// ---------------------------------------------------------------- MC step
// One MonteCarlo::apply iteration (sampling.cc:55-99) on one stream: the fold
// launches of the walkers whose sequence changed (launch_window) between two
// runs of step_tail_kernel, one wave per walker: the Metropolis decision of
// the step before (accept_walker) and the next proposal (propose_walker:
// thermostat, RNG streams, mutation move, unchanged check) with its fold's
// weight class (fold_class, for order_kernel).  The MC state stays out of the
// fold kernels' register allocation.

// What a tail reads that nothing in it writes, loaded in one batch at its top
// (the decision's and the proposal's chains then wait on LDS and on the
// move tables only)
struct TailIn {
    int err = 0, changed = 0, ovf = 0, tabv = 0;
    double ps = 0.0, cs = 0.0, temp = 1.0, u = 0.0;
    int ia = 624, ic = 624;   // MT stream indices
    int ntrain = 0;
    double auto_T = 0.0, last_diff = 0.0;
};

struct Accepted {
    bool ran = false;       // a decision was taken (no move error)
    bool changed = false;   // the proposal was scored: last_diff = diff
    bool took = false;      // accepted: the proposal is the current sequence
    double diff = 0.0;
    int tab_valid = -1;     // >= 0: the walker's new tab_valid
};

// Metropolis (sampling.cc:76-89).  cur_slot / tab_valid (null without stored
// tables): an accepted proposal's tables become current, and complete (every
// kernel writes the whole slot), so a walker whose current tables were invalid
// (imported configuration, MFE fold outside the 16-bit range) refolds
// incrementally again -- unless this very fold left the 16-bit range (ovf,
// MFE: its slot is not exact).  Every lane takes the (uniform) decision, lane 0
// writes the walker's state; the accepted sequence is copied by the tail.
// kc (comb set): the step's fold launches left the proposal's score as
// per-variant energies (KArgs::defer_comb): combined here (combine_wave) and
// stored, but for an MFE fold the FP32 fallback redid (ovf; it stored the score).
__device__ Accepted accept_walker(const StepArgs &st, const KArgs &kc, bool comb, double *tv, int w, int lane, int s,
                                  int nt_tot, const TailIn &in) {
    Accepted a;
    if (in.err) return a;
    a.ran = true;
    const bool changed = in.changed == 1;
    int outcome = 2;  // ACCEPT_UNCHANGED
    double prop = in.ps;
    if (changed && comb && !in.ovf) {
        prop = combine_wave(kc, w, lane, tv ? tv + size_t(w) * nt_tot : nullptr);
        if (lane == 0) st.prop_score[w] = prop;
    }
    double diff = 0.0;
    if (changed) {
        diff = prop - in.cs;
        const double crit = exp(diff / in.temp);
        outcome = (crit < in.u) ? 0 : (diff > 0) ? 3 : 1;
    }
    a.changed = changed;
    a.diff = diff;
    const bool acc = outcome == 1 || outcome == 3;
    a.took = acc;
    if (acc && st.cur_slot) a.tab_valid = in.ovf ? 0 : 1;
    if (lane == 0) {
        if (changed) st.last_diff[w] = diff;
        if (acc) {
            st.cur_score[w] = prop;
            if (st.cur_slot) {
                st.cur_slot[w] ^= 1;   // the proposal's tables become current
                st.tab_valid[w] = uint8_t(a.tab_valid);
            }
        }
        st.counters[size_t(w) * 4 + outcome] += 1;
        if (st.tr_pos) {
            const size_t r = size_t(s) * st.W + w;
            st.tr_outcome[r] = outcome;
            st.tr_prop[r] = changed ? prop : __builtin_nan("");
            st.tr_cur[r] = acc ? prop : in.cs;
            st.tr_u[r] = changed ? in.u : __builtin_nan("");
            if (!changed && st.tr_terms)
                for (int k = 0; k < nt_tot; k++) st.tr_terms[r * nt_tot + k] = __builtin_nan("");
        }
    }
    return a;
}

struct Proposed {
    bool scored = false;    // the fold launch scores this walker
    int plo = -1, phi = -1;
};

// The proposal of step `step` (trace row s).  seq: the walker's current
// sequence, staged in LDS by the tail (the proposal of the step before when
// acc took it); acc's score difference is the auto thermostat's training
// value.  a, c: the streams, their next words staged by the tail (MtView).
__device__ Proposed propose_walker(const StepArgs &st, long long step, int s, int w, int lane, const Accepted &acc,
                                   const TailIn &in, const uint8_t *seq, MtView &a, MtView &c) {
    Proposed out;
    if (in.err) {
        if (lane == 0) st.changed[w] = 0;
        return out;
    }
    uint8_t *prop = st.prop_seq + size_t(w) * st.Nraw;
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
        const int n = in.ntrain + 1;
        T = in.auto_T;
        double Tn = T;
        if (lane == 0) {
            tr[n - 1] = acc.changed ? acc.diff : in.last_diff;
            if (n >= st.period) {
                // median = std::nth_element at n/2, clamp = std::max(t, 0.0)
                // (sampling.cc:389-396): the libstdc++ selection, so -0.0 / NaN
                // land exactly where the reference's do
                const int k = n / 2;
                nth_element_libstdcxx(tr, k, n);
                const double t = tr[k] / st.ln_target_rate;
                Tn = (t < 0.0) ? 0.0 : t;
                st.auto_T[w] = Tn;
                st.ntrain[w] = 0;
            } else {
                st.ntrain[w] = n;
            }
        }
        T = __shfl(Tn, 0, WAVE);
    }
    // ---- move: stream A (and C if the step will be scored)
    const int pick = int(mt_uniform(a, uint32_t(st.M), lane));
    const int bcode = int(mt_uniform(a, 4u, lane)) + 1;  // "ACGU"[r]
    const int e = st.clo_err[pick];
    const int k0 = st.clo_off[pick], k1 = st.clo_off[pick + 1];
    bool changed = false;
    int plo = 1 << 30, phi = -1;   // hull of the positions whose base changes (incremental folds)
    if (e == 0) {
        for (int k = k0 + lane; k < k1; k += WAVE) {
            const int pos = st.clo_pos[k];
            const int nb = st.clo_par[k] ? 5 - bcode : bcode;
            if (seq[pos] != nb) {
                changed = true;
                plo = min(plo, pos);
                phi = max(phi, pos);
            }
        }
        changed = __ballot(changed) != 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            plo = min(plo, __shfl_xor(plo, o, WAVE));
            phi = max(phi, __shfl_xor(phi, o, WAVE));
        }
    }
    double u = 0.0;
    if (e == 0 && changed) u = mt_canonical(c, lane);
    if (a.twisted)
        for (int k = lane; k < 624; k += WAVE) gA[k] = a.mt[k];
    if (c.twisted)
        for (int k = lane; k < 624; k += WAVE) gC[k] = c.mt[k];
    if (changed) {
        // the proposal: the staged sequence with the move's positions replaced
        for (int k = lane; k < st.Nraw; k += WAVE) {
            uint8_t b = seq[k];
            for (int q = k0; q < k1; q++)
                if (st.clo_pos[q] == k) b = uint8_t(st.clo_par[q] ? 5 - bcode : bcode);
            prop[k] = b;
        }
    }
    if (lane == 0) {
        gA[624] = uint32_t(a.idx);
        gC[624] = uint32_t(c.idx);
        st.pick[w] = pick;
        st.bcode[w] = bcode;
        st.temp[w] = T;
        st.u[w] = u;
        st.changed[w] = (e != 0) ? 0 : (changed ? 1 : 0);
        if (st.chg) {
            st.chg[2 * w] = changed ? plo : -1;
            st.chg[2 * w + 1] = changed ? phi : -1;
        }
        if (e != 0) st.err[w] = e;
        if (st.tr_pos) {
            const size_t r = size_t(s) * st.W + w;
            st.tr_pos[r] = st.mut[pick];
            st.tr_base[r] = int8_t(bcode);
            st.tr_temp[r] = T;
        }
    }
    out.scored = e == 0 && changed;
    out.plo = changed ? plo : -1;
    out.phi = changed ? phi : -1;
    return out;
}

// The weight class of a proposal's fold for the launch order (order_kernel):
// 0 = heaviest .. 63 by the band of cells containing a changed position, about
// (m_hi + 2) (N - m_lo + 1), a fold from scratch (no valid stored tables)
// counting as the whole triangle; 64 = not scored.
__device__ __forceinline__ int fold_class(const StepArgs &st, const Proposed &p, int tabv) {
    if (!p.scored) return 64;
    const long long full = (long long)st.Nraw * st.Nraw;
    long long key = full;
    if (tabv && st.chg && p.plo >= 0) key = (long long)(p.phi + 2) * (st.Nraw - p.plo + 1);
    return 63 - int(min(full, max(0LL, key)) * 63 / (full > 0 ? full : 1));
}

// One wave per walker: the decision of step s_acc (< 0: none, the first
// proposal of a launch; comb, tv: accept_walker) and the proposal of global
// step `step` (< 0: none, the last step of a launch; trace row s_prop).
// Across a launch_steps call the two halves of a step meet only through HBM
// written by the launches between.  The walker's scalars, its current and
// proposed sequences and its MT streams' next words are loaded in one batch
// first; the sequence the proposal starts from is staged in LDS.
constexpr int TAIL_NMAX = 256;   // sequences staged whole
static_assert(NMAX < TAIL_NMAX, "adx_api limits sequences to NMAX: the step tail stages them whole");
constexpr int TAIL_WPB = 4;      // walkers (waves) per workgroup
__global__ void __launch_bounds__(TAIL_WPB * 64) step_tail_kernel(StepArgs st, KArgs kc, int comb, double *tv,
                                                                  int s_acc, long long step, int s_prop, int nt_tot) {
    __shared__ uint32_t mts[TAIL_WPB][2 * MT_WORDS];
    __shared__ uint8_t seqs[TAIL_WPB][TAIL_NMAX];
    const int wv = int(threadIdx.x) >> 6;
    const int w = int(blockIdx.x) * TAIL_WPB + wv;
    const int lane = int(threadIdx.x) & (WAVE - 1);
    if (w >= st.W) return;   // no workgroup barrier below: each wave owns its walker and LDS
    uint32_t *mt = mts[wv];
    uint8_t *seq = seqs[wv];
    const int Nr = st.Nraw;
    uint32_t *gA = st.mtA + size_t(w) * MT_WORDS;
    uint32_t *gC = st.mtC + size_t(w) * MT_WORDS;
    const uint8_t *curg = st.cur_seq + size_t(w) * Nr, *propg = st.prop_seq + size_t(w) * Nr;
    TailIn in;
    in.err = st.err[w];
    in.changed = st.changed[w];
    in.ps = st.prop_score[w];
    in.cs = st.cur_score[w];
    in.temp = st.temp[w];
    in.u = st.u[w];
    in.ovf = st.ovf ? st.ovf[w] : 0;
    in.tabv = st.tab_valid ? st.tab_valid[w] : 0;
    in.ia = int(gA[624]);
    in.ic = int(gC[624]);
    if (st.thermo_kind == 2) {
        in.ntrain = st.ntrain[w];
        in.auto_T = st.auto_T[w];
        in.last_diff = st.last_diff[w];
    }
    constexpr int SP = TAIL_NMAX / WAVE;   // bytes a lane holds, packed (position q * 64 + lane in byte q)
    uint32_t cb = 0, pb = 0;
#pragma unroll
    for (int q = 0; q < SP; q++) {
        const int k = q * WAVE + lane;
        cb |= uint32_t(k < Nr ? curg[k] : 0) << (8 * q);
        pb |= uint32_t((k < Nr && s_acc >= 0) ? propg[k] : 0) << (8 * q);
    }
    // the streams' next 8 words (a step draws 2 + 2 but for a rejection: past
    // the window MtView reads HBM, at a twist it stages the whole state)
    if (step >= 0) {
        if (lane < 8) {
            if (in.ia + lane < 624) mt[in.ia + lane] = gA[in.ia + lane];
        } else if (lane < 16) {
            if (in.ic + lane - 8 < 624) mt[MT_WORDS + in.ic + lane - 8] = gC[in.ic + lane - 8];
        }
    }
    Accepted acc;
    if (s_acc >= 0) {
        acc = accept_walker(st, kc, comb != 0, tv, w, lane, s_acc, nt_tot, in);
        if (acc.took) {   // the proposal becomes the current sequence
            uint8_t *c = st.cur_seq + size_t(w) * Nr;
#pragma unroll
            for (int q = 0; q < SP; q++) {
                const int k = q * WAVE + lane;
                if (k < Nr) c[k] = uint8_t(pb >> (8 * q));
            }
        }
    }
    if (step < 0) return;
#pragma unroll
    for (int q = 0; q < SP; q++) {
        const int k = q * WAVE + lane;
        if (k < Nr) seq[k] = uint8_t((acc.took ? pb : cb) >> (8 * q));
    }
    wave_sync();
    MtView a{mt, gA, in.ia, in.ia, min(in.ia + 8, 624), false};
    MtView c{mt + MT_WORDS, gC, in.ic, in.ic, min(in.ic + 8, 624), false};
    const Proposed p = propose_walker(st, step, s_prop, w, lane, acc, in, seq, a, c);
    if (lane == 0) {
        if (st.ovf) st.ovf[w] = 0;   // set again by this proposal's fold if it leaves the 16-bit range
        if (st.cls) st.cls[w] = uint8_t(fold_class(st, p, acc.tab_valid >= 0 ? acc.tab_valid : in.tabv));
    }
}

}  // namespace

// ---------------------------------------------------------------- host launchers
// P = 2 (apo/holo lockstep, 16 waves) when its LDS fits one CU, else P = 1
// (8 waves, two workgroups per CU when they fit).
#ifndef ADX_NT2
#define ADX_NT2 768     // 12 waves x 168 VGPRs (16 x 128 spills)
#endif
#define ADX_STR_(x) #x
#define ADX_STR(x) ADX_STR_(x)
#ifndef ADX_NT16
#define ADX_NT16 512    // packed 16-bit MFE
#endif
template <int P, int NT = (P == 2 ? ADX_NT2 : 512)>
static size_t lds_size(const KArgs &ka, int pl, bool rt) {
    return lds_layout<true, P>(nullptr, ka.cells, ka.Nmax, ka.n_variants, nullptr, pl, rt, NT / WAVE);
}

static int choose_p(const KArgs &ka) {
    return lds_size<2>(ka, 0, false) <= size_t(LDS_LIMIT) ? 2 : 1;
}

// optional LDS arrays (rank list, range table) when they still fit
template <int P, int NT = (P == 2 ? ADX_NT2 : 512)>
static void choose_opt(const KArgs &ka, int &pl, bool &rt) {
    // P = 1 keeps two workgroups per CU when they fit (1 KiB margin for allocation granularity)
    const size_t lim = (P == 1 && 2 * lds_size<1, NT>(ka, 0, false) <= size_t(LDS_LIMIT) - 2048)
                           ? LDS_LIMIT / 2 - 1024 : LDS_LIMIT;
    rt = lds_size<P, NT>(ka, 0, true) <= lim;
    pl = lds_size<P, NT>(ka, 2, rt) <= lim ? 2 : lds_size<P, NT>(ka, 1, rt) <= lim ? 1 : 0;
}

size_t lds_bytes(const KArgs &ka, bool /*unused*/, int /*nt*/) {
    int pl;
    bool rt;
    if (choose_p(ka) == 2) {
        choose_opt<2>(ka, pl, rt);
        return lds_size<2>(ka, pl, rt);
    }
    choose_opt<1>(ka, pl, rt);
    return lds_size<1>(ka, pl, rt);
}

template <int NT, int P, class SR>
static hipError_t launch_score_t(const KArgs &ka, const uint8_t *seqs, int W, double *scores, double *terms,
                                 float *dG, const int *mask, hipStream_t stream, int grid = 0) {
    int pl;
    bool rt;
    choose_opt<P, NT>(ka, pl, rt);
    const size_t lds = lds_size<P, NT>(ka, pl, rt);
    auto k = score_kernel<NT, P, SR>;
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    KArgs kb = ka;
    kb.opt = pl | (rt ? 4 : 0);
    hipLaunchKernelGGL(k, dim3(grid > 0 && grid < W ? grid : W), dim3(NT), lds, stream, kb, kb.X, seqs, W, scores,
                       terms, dG, mask);
    return hipGetLastError();
}

// Scores from the per-variant energies a fold kernel left in KArgs::gstep
// (combine_score, one thread per walker): after pf_cells_kernel, and after the
// outside pass once it has written the pair probabilities (pair_p null: the
// pair terms read 0.5, as combine_score).
__global__ void combine_kernel(KArgs ka, int W, const int *mask, double *scores, double *terms) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W || (mask && mask[w] != 1)) return;
    const float *g = ka.gstep + size_t(w) * ka.n_variants;
    const double *pp = ka.pair_p ? ka.pair_p + size_t(w) * ka.n_pairs : nullptr;
    const int nt = ka.n_terms * ka.n_ctx_eff;
    double *tv = terms ? terms + size_t(w) * nt : nullptr;
    double score = 0.0;
    for (int idx = 0; idx < nt; idx++) {
        double wt;
        const double val = term_value(ka, g, pp, idx, wt);
        if (tv) tv[idx] = val;
        score += wt * val;
    }
    scores[w] = score;
}

size_t mfe_cells_lds(const KArgs &ka);
size_t pf_cells_lds(const KArgs &ka);
hipError_t launch_pf_ring(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, float *gout,
                          float *qscr, hipStream_t stream);
hipError_t launch_pf_cells(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, float *gout,
                           hipStream_t stream);
hipError_t launch_mfe_cells(const KArgs &ka, const uint8_t *seqs, int W, float *gout, const int *mask,
                            hipStream_t stream);
bool mfe_pair_active(const KArgs &ka);

// MFE kernel choice, ADX_MFE_KERNEL (read at every launch, so a test can
// switch it between contexts): cells (default) = mfe_cells_kernel (lanes =
// cells, two folds per cell, two walkers per CU); rows = score_kernel<MinPlus16>
// (lanes = terms) -- also the kernel for energy models or lengths the cells
// kernel does not cover (mfe_cells_lds() == 0)
static bool mfe_rows_forced() {
    const char *e = std::getenv("ADX_MFE_KERNEL");
    return e && std::strcmp(e, "rows") == 0;
}
static bool pf_rows_forced() {
    const char *e = std::getenv("ADX_PF_KERNEL");
    return e && std::strcmp(e, "rows") == 0;
}

// The fold kernel launch_score_m runs for a workload (one choice, used by the
// dispatch and by the names the bench reports)
enum class InsideK { MfeCells, MfeRows16, MinPlusP2, MinPlus512, PfCells, PfRing, SumProdP2, SumProd768, SumProd512 };
static InsideK inside_choice(const KArgs &ka, bool has_g) {
    // ka.mode: 0 = partition functions (vrna_pf), 1 = minimum free energies
    if (ka.mode == 1 && ka.X16 && ka.ovf) {
        KArgs k16 = ka;
        k16.T = ka.T16;
        k16.X = ka.X16;
        return (!mfe_rows_forced() && mfe_cells_lds(k16) > 0) ? InsideK::MfeCells : InsideK::MfeRows16;
    }
    if (ka.mode == 1) return choose_p(ka) == 2 ? InsideK::MinPlusP2 : InsideK::MinPlus512;
    if (ka.pf_ring) return InsideK::PfRing;   // the context's slot layout (adx_api.cpp upload_all)
    if (has_g && !pf_rows_forced() && choose_p(ka) == 2 && ka.n_groups2 > 0 && pf_cells_lds(ka) > 0)
        return InsideK::PfCells;
    if (choose_p(ka) == 2) return InsideK::SumProdP2;
    // one workgroup per CU (N = 150: the P = 1 tables take most of the LDS): 12
    // waves instead of 8, 168 VGPRs a lane (16 waves at 128 spill: 29.9 vs 28.2 ms)
    if (2 * lds_size<1, 512>(ka, 0, false) > size_t(LDS_LIMIT) - 2048) return InsideK::SumProd768;
    return InsideK::SumProd512;
}

const char *inside_kernel_name(const KArgs &ka) {
    switch (inside_choice(ka, ka.gstep != nullptr)) {
        case InsideK::MfeCells: {
            KArgs k16 = ka;
            k16.T = ka.T16;
            k16.X = ka.X16;
            return mfe_pair_active(k16) ? "mfe_pair_kernel + score_kernel<MinPlus> (FP32 fallback launch); scores combined in step_tail_kernel"
                                        : "mfe_cells_kernel + score_kernel<MinPlus> (FP32 fallback launch); scores combined in step_tail_kernel";
        }
        case InsideK::MfeRows16: return "score_kernel<" ADX_STR(ADX_NT16) ", 1, MinPlus16> + score_kernel<MinPlus> (FP32 fallback launch)";
        case InsideK::MinPlusP2: return "score_kernel<" ADX_STR(ADX_NT2) ", 2, MinPlus>";
        case InsideK::MinPlus512: return "score_kernel<512, 1, MinPlus>";
        case InsideK::PfCells: return "pf_cells_kernel (scores combined in step_tail_kernel)";
        case InsideK::PfRing: return "pf_ring_kernel (scores combined in step_tail_kernel)";
        case InsideK::SumProdP2: return "score_kernel<" ADX_STR(ADX_NT2) ", 2, SumProd>";
        case InsideK::SumProd768: return "score_kernel<768, 1, SumProd>";
        default: return "score_kernel<512, 1, SumProd>";
    }
}

hipError_t launch_score_m(const KArgs &ka, const uint8_t *seqs, int W, double *scores, double *terms,
                          float *dG, const int *mask, hipStream_t stream) {
    float *g = dG ? dG : ka.gstep;
    const InsideK k = inside_choice(ka, g != nullptr);
    if (k == InsideK::MfeCells || k == InsideK::MfeRows16) {
        // packed 16-bit folds (two variants per value, two workgroups per CU), then
        // the FP32 MinPlus kernel for the walkers whose values left the exact range
        KArgs k16 = ka;
        k16.T = ka.T16;
        k16.X = ka.X16;
        hipError_t e;
        if (k == InsideK::MfeCells) {
            // one workgroup per (walker, fold group): energies to dG (or the gstep
            // scratch), then the scores (the same arithmetic as combine_score)
            if (!g) return hipErrorInvalidValue;
            e = launch_mfe_cells(k16, seqs, W, g, mask, stream);
            if (e == hipSuccess && !(ka.defer_comb && mask)) {
                KArgs kc = ka;
                kc.gstep = g;
                hipLaunchKernelGGL(combine_kernel, dim3((W + 255) / 256), dim3(256), 0, stream, kc, W, mask, scores,
                                   terms);
                e = hipGetLastError();
            }
        } else {
            e = launch_score_t<ADX_NT16, 1, MinPlus16>(k16, seqs, W, scores, terms, dG, mask, stream);
        }
        if (e != hipSuccess) return e;
        KArgs kf = ka;            // the FP32 fallback folds from scratch, keeps no state
        kf.tab = nullptr;
        // overflows are rare: one block per CU scans the flags (ovf) instead of W
        // blocks that mostly exit at once
#ifndef ADX_FB_GRID
#define ADX_FB_GRID 64
#endif
        constexpr int FB_GRID = ADX_FB_GRID;
        if (choose_p(ka) == 2)
            return launch_score_t<ADX_NT2, 2, MinPlus>(kf, seqs, W, scores, terms, dG, ka.ovf, stream, FB_GRID);
        return launch_score_t<512, 1, MinPlus>(kf, seqs, W, scores, terms, dG, ka.ovf, stream, FB_GRID);
    }
    switch (k) {
        case InsideK::MinPlusP2: return launch_score_t<ADX_NT2, 2, MinPlus>(ka, seqs, W, scores, terms, dG, mask, stream);
        case InsideK::MinPlus512: return launch_score_t<512, 1, MinPlus>(ka, seqs, W, scores, terms, dG, mask, stream);
        case InsideK::PfCells: {
            // lanes = cells (pf_cells.hip): energies to dG (or the gstep scratch), then the scores
            hipError_t e = launch_pf_cells(ka, seqs, W, mask, g, stream);
            if (e != hipSuccess) return e;
            if (ka.defer_comb && mask) return hipSuccess;   // the step's tail combines
            KArgs kc = ka;
            kc.gstep = g;
            hipLaunchKernelGGL(combine_kernel, dim3((W + 255) / 256), dim3(256), 0, stream, kc, W, mask, scores, terms);
            return hipGetLastError();
        }
        case InsideK::PfRing: {
            // one workgroup per variant, qb ring (pf_ring.hip), then the scores
            if (!g) return hipErrorInvalidValue;
            hipError_t e = launch_pf_ring(ka, seqs, W, mask, g, ka.tab ? nullptr : ka.ring_scratch, stream);
            if (e != hipSuccess) return e;
            if (ka.defer_comb && mask) return hipSuccess;   // the step's tail combines
            KArgs kc = ka;
            kc.gstep = g;
            hipLaunchKernelGGL(combine_kernel, dim3((W + 255) / 256), dim3(256), 0, stream, kc, W, mask, scores, terms);
            return hipGetLastError();
        }
        case InsideK::SumProdP2: return launch_score_t<ADX_NT2, 2, SumProd>(ka, seqs, W, scores, terms, dG, mask, stream);
        case InsideK::SumProd768: return launch_score_t<768, 1, SumProd>(ka, seqs, W, scores, terms, dG, mask, stream);
        default: return launch_score_t<512, 1, SumProd>(ka, seqs, W, scores, terms, dG, mask, stream);
    }
}

hipError_t launch_score(const KArgs &ka, bool, const uint8_t *seqs, int W, double *scores,
                        double *terms, float *dG, hipStream_t stream) {
    return launch_score_m(ka, seqs, W, scores, terms, dG, nullptr, stream);
}

// outside pass: LDS bytes of the all-LDS layout, or of the global-scratch
// layout (gout = true) when that does not fit; 0 when neither fits one CU.
size_t bppm_lds_bytes(const KArgs &ka, bool *gout) {
    const size_t o = lds_layout<true, 1>(nullptr, ka.cells, ka.Nmax, ka.n_variants, nullptr, 0, false);
    const size_t t = outs_layout<true, false>(nullptr, o, ka.cells, ka.Nmax, nullptr);
    if (t <= size_t(LDS_LIMIT)) {
        if (gout) *gout = false;
        return t;
    }
    const size_t tg = outs_layout<true, true>(nullptr, o, ka.cells, ka.Nmax, nullptr);
    if (gout) *gout = true;
    return tg <= size_t(LDS_LIMIT) ? tg : 0;
}
size_t bppm_scratch_bytes(const KArgs &ka, int W) {
    bool gout = false;
    if (bppm_lds_bytes(ka, &gout) == 0 || !gout) return 0;
    return size_t(W) * ka.n_bvars * outs_global_bytes(ka.cells);
}

template <bool GOUT>
static hipError_t launch_bppm_t(const KArgs &ka, size_t lds, const uint8_t *seqs, int W, const int *mask,
                                double *full, int ld, double *pair_p, char *scratch, hipStream_t stream,
                                bool reuse) {
    auto k = bppm_kernel<GOUT ? 1024 : 512, GOUT>;   // GOUT (N = 150): one workgroup per CU, 16 waves (12: 50.1 vs 49.1 ms)
    static size_t configured = 0;
    if (lds > configured) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
        configured = lds;
    }
    hipLaunchKernelGGL(k, dim3(W * ka.n_bvars), dim3(GOUT ? 1024 : 512), lds, stream, ka, ka.X, seqs, W, mask, full, ld, pair_p,
                       scratch, choose_p(ka), reuse ? 1 : 0);
    return hipGetLastError();
}

static hipError_t launch_bppm_r(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *full, int ld,
                                double *pair_p, char *scratch, hipStream_t stream, bool reuse) {
    bool gout = false;
    const size_t lds = bppm_lds_bytes(ka, &gout);
    if (lds == 0 || ka.n_bvars <= 0 || (gout && !scratch)) return hipErrorInvalidValue;
    if (gout) return launch_bppm_t<true>(ka, lds, seqs, W, mask, full, ld, pair_p, scratch, stream, reuse);
    return launch_bppm_t<false>(ka, lds, seqs, W, mask, full, ld, pair_p, nullptr, stream, reuse);
}

size_t outside_cells_lds(const KArgs &ka);
hipError_t launch_outside_cells(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *pair_p,
                                int sp_score, hipStream_t stream);

// The outside pass of an MC step with pair terms (launch_steps): the lanes =
// cells kernel where it covers the workload, else bppm_kernel on the stored
// tables (ADX_OUTSIDE_KERNEL=bppm forces the latter)
size_t outside_ring_lds(const KArgs &ka);
hipError_t launch_outside_ring(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *pair_p,
                               hipStream_t stream);
static bool outside_is_cells(const KArgs &ka) {
    if (ka.pf_ring) return false;   // the ring's slot layout: outside_ring_kernel
    const char *ok = std::getenv("ADX_OUTSIDE_KERNEL");
    const bool old = ok && std::strcmp(ok, "bppm") == 0;
    return !old && outside_cells_lds(ka) > 0;
}
const char *outside_kernel_name(const KArgs &ka) {
    if (ka.n_pairs <= 0) return "";
    if (!(ka.mode == 0 && ka.tab && ka.gstep)) {   // launch_steps' fallback branch: bppm from scratch
        bool gout = false;
        bppm_lds_bytes(ka, &gout);
        return gout ? "bppm_kernel<1024, GOUT> (inside refold + outside)" : "bppm_kernel<512> (inside refold + outside)";
    }
    if (ka.pf_ring) return "outside_ring_kernel";
    if (outside_is_cells(ka)) return "outside_cells_kernel";
    bool gout = false;
    bppm_lds_bytes(ka, &gout);
    return gout ? "bppm_kernel<1024, GOUT>" : "bppm_kernel<512>";
}

// scratch: bppm_scratch_bytes(ka, W) bytes of device memory (null when 0)
hipError_t launch_bppm(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *full, int ld,
                       double *pair_p, char *scratch, hipStream_t stream) {
    return launch_bppm_r(ka, seqs, W, mask, full, ld, pair_p, scratch, stream, false);
}

// Launch order of an MC step's folds: the walkers whose proposal is scored,
// heaviest refold first, then the unscored ones (their blocks exit at once) --
// a counting sort of the weight classes the proposals computed (fold_class;
// a rescore's are all 0).  The folds' durations vary by several times and the
// GPU starts workgroups in launch order, so heavy folds no longer trail the
// launch.  One workgroup, LDS counters, the class bases by one wave's scan;
// the order within a class does not matter (each walker's fold is independent
// of where it runs).
__global__ void __launch_bounds__(1024) order_kernel(int W, const uint8_t *cls, int *order) {
    __shared__ int hist[65];
    const int tid = threadIdx.x;
    if (tid < 65) hist[tid] = 0;
    __syncthreads();
#pragma unroll 4
    for (int w = tid; w < W; w += 1024) atomicAdd(&hist[cls[w]], 1);
    __syncthreads();
    if (tid < WAVE) {   // exclusive scan of classes 0..63; the unscored (64) after them
        const int h = hist[tid];
        int incl = h;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const int t = __shfl_up(incl, o, WAVE);
            if (tid >= o) incl += t;
        }
        hist[tid] = incl - h;
        if (tid == WAVE - 1) hist[64] = incl;
    }
    __syncthreads();
#pragma unroll 4
    for (int w = tid; w < W; w += 1024) order[atomicAdd(&hist[cls[w]], 1)] = w;
}

// Whether launch_window leaves a step's scores as energies in gstep (KArgs::
// defer_comb set): the fold kernels that write per-variant energies and the
// outside pass of the pair terms
static bool window_defers(const KArgs &ka) {
    if (!ka.defer_comb) return false;
    if (ka.n_pairs > 0 && ka.mode == 0 && ka.tab && ka.gstep) return true;
    const InsideK k = inside_choice(ka, ka.gstep != nullptr);
    return k == InsideK::MfeCells || k == InsideK::PfCells || k == InsideK::PfRing;
}

// The score window of one MC step for the walkers flagged in `changed`: the
// proposals' folds (prop_seq; incremental against the stored tables where
// tab_valid allows), the outside pass when terms read base-pair probabilities,
// the scores (prop_score) and term values (tv, optional).  evs (optional, 4):
// window start, outside pass start, outside pass end, window end.
static hipError_t launch_window(const KArgs &ka, const StepArgs &st, const int *changed, double *tv,
                                hipStream_t stream, hipEvent_t *evs) {
    if (evs) (void)hipEventRecord(evs[0], stream);
    if (ka.order) hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, stream, st.W, ka.ocls, ka.order);
    hipError_t e;
    if (ka.n_pairs > 0 && ka.mode == 0 && ka.tab && ka.gstep) {
        // inside folds first (they write the proposal's tables), then the outside
        // pass on those tables, then the scores with the pair probabilities
        KArgs ki = ka;
        ki.pair_p = nullptr;
        e = launch_score_m(ki, st.prop_seq, st.W, st.prop_score, nullptr, ka.gstep, changed, stream);
        if (e != hipSuccess) return e;
        if (evs) (void)hipEventRecord(evs[1], stream);
        // lanes = cells outside kernel (outside_cells.hip) where it covers the
        // length, else bppm_kernel on the same stored tables
        e = ka.pf_ring ? launch_outside_ring(ka, st.prop_seq, st.W, changed, const_cast<double *>(ka.pair_p),
                                             stream)
            : outside_is_cells(ka)
                ? launch_outside_cells(ka, st.prop_seq, st.W, changed, const_cast<double *>(ka.pair_p),
                                       choose_p(ka), stream)
                : launch_bppm_r(ka, st.prop_seq, st.W, changed, nullptr, 0, const_cast<double *>(ka.pair_p),
                                ka.bppm_scratch, stream, true);
        if (e != hipSuccess) return e;
        if (evs) (void)hipEventRecord(evs[2], stream);
        if (!ka.defer_comb) {
            hipLaunchKernelGGL(combine_kernel, dim3((st.W + 255) / 256), dim3(256), 0, stream, ka, st.W, changed,
                               st.prop_score, tv);
            e = hipGetLastError();
        }
    } else {
        // events 1 / 2 bracket the outside pass (here before the folds; none: empty)
        if (evs) (void)hipEventRecord(evs[1], stream);
        if (ka.n_pairs > 0) {   // base-pair probabilities the score terms read (outside pass)
            e = launch_bppm(ka, st.prop_seq, st.W, changed, nullptr, 0, const_cast<double *>(ka.pair_p),
                            ka.bppm_scratch, stream);
            if (e != hipSuccess) return e;
        }
        if (evs) (void)hipEventRecord(evs[2], stream);
        e = launch_score_m(ka, st.prop_seq, st.W, st.prop_score, tv, nullptr, changed, stream);
    }
    if (evs) (void)hipEventRecord(evs[3], stream);
    return e;
}

// evs (optional): 4 * nsteps events per step: window start, outside pass
// start, outside pass end, window end (score written); the inside share of a
// window is the window minus its outside pass (adx_api.cpp).  Launches:
// step_tail_kernel (the first proposals), then per step the score window and
// step_tail_kernel (its decisions and the next step's proposals).
hipError_t launch_steps(const KArgs &ka, bool, const StepArgs &st0, hipStream_t stream, hipEvent_t *evs) {
    const int nt_tot = ka.n_terms * ka.n_ctx_eff;
    if (st0.nsteps <= 0) return hipSuccess;   // (the first tail would draw a proposal)
    StepArgs st = st0;
    st.cur_slot = ka.tab ? ka.cur_slot : nullptr;
    st.tab_valid = ka.tab ? ka.tab_valid : nullptr;
    st.ovf = ka.mode == 1 ? ka.ovf : nullptr;
    st.cls = ka.order ? const_cast<uint8_t *>(ka.ocls) : nullptr;   // ordering off: ADX_NO_ORDER / no stored tables
    const dim3 tg((st.W + TAIL_WPB - 1) / TAIL_WPB), tb(TAIL_WPB * 64);
    hipLaunchKernelGGL(step_tail_kernel, tg, tb, 0, stream, st, ka, 0, (double *)nullptr, -1, st.step0, 0, nt_tot);
    KArgs kas = ka;
    kas.defer_comb = 1;   // the tails combine the scores the windows leave as energies
    const int comb = window_defers(kas) ? 1 : 0;
    for (int s = 0; s < st.nsteps; s++) {
        double *tv = st.tr_terms ? st.tr_terms + size_t(s) * st.W * nt_tot : nullptr;
        hipError_t e = launch_window(kas, st, st.changed, tv, stream, evs ? evs + 4 * s : nullptr);
        if (e != hipSuccess) return e;
        const bool more = s + 1 < st.nsteps;
        hipLaunchKernelGGL(step_tail_kernel, tg, tb, 0, stream, st, kas, comb, tv, s, more ? st.step0 + s + 1 : -1LL,
                           s + 1, nt_tot);
    }
    return hipGetLastError();
}

__global__ void rescore_begin_kernel(int W, int *changed, uint8_t *tab_valid, uint8_t *cls, int *ovf) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    changed[w] = 1;
    if (tab_valid) tab_valid[w] = 0;
    if (cls) cls[w] = 0;   // folds from scratch: one weight class
    if (ovf) ovf[w] = 0;
}

__global__ void rescore_end_kernel(int W, uint8_t *cur_slot, uint8_t *tab_valid, const int *ovf) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    // the fresh tables of the (unchanged) current sequence are in the other slot;
    // an MFE fold that left the 16-bit range (re-folded in FP32) wrote none
    cur_slot[w] = uint8_t(1 - cur_slot[w]);
    tab_valid[w] = (ovf && ovf[w]) ? 0 : 1;
}

// Every walker's current configuration folded and scored FROM SCRATCH with the
// MC step's own kernels (launch_window: the same inside, outside and combine
// launches, tables written to the walker's other slot and then adopted): the
// walkers' first scores (adx_walkers_init) and adx_walkers_rescore, so stored
// scores, incremental refolds and a fresh fold agree bit for bit.  Scores land
// in st.prop_score (tv: term values, optional); no move, no Metropolis.
hipError_t launch_rescore(const KArgs &ka, const StepArgs &st, double *tv, hipStream_t stream) {
    hipError_t e = hipMemcpyAsync(st.prop_seq, st.cur_seq, size_t(st.W) * st.Nraw, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return e;
    const dim3 g((st.W + 255) / 256), b(256);
    hipLaunchKernelGGL(rescore_begin_kernel, g, b, 0, stream, st.W, st.changed, ka.tab ? ka.tab_valid : nullptr,
                       ka.order ? const_cast<uint8_t *>(ka.ocls) : nullptr, ka.mode == 1 ? ka.ovf : nullptr);
    e = launch_window(ka, st, st.changed, tv, stream, nullptr);
    if (e != hipSuccess) return e;
    if (ka.tab)
        hipLaunchKernelGGL(rescore_end_kernel, g, b, 0, stream, st.W, ka.cur_slot, ka.tab_valid,
                           ka.mode == 1 ? ka.ovf : nullptr);
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
