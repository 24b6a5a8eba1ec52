// C ABI of the MI355X engine (include/addapt_gpu.h): run setup on the host,
// device buffers, kernel launches.  The reference's objects this replaces are
// cited per function; the heavy lifting is in kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/addapt_gpu.h"
#include "dev_types.hpp"
#include "energy.hpp"

namespace adx {
size_t lds_bytes(const KArgs &ka, bool qbm, int nt);
hipError_t launch_score(const KArgs &ka, bool qbm, const uint8_t *seqs, int W, double *scores,
                        double *terms, float *dG, hipStream_t stream);
hipError_t launch_steps(const KArgs &ka, bool qbm, const StepArgs &st, hipStream_t stream, hipEvent_t *evs);
hipError_t launch_rescore(const KArgs &ka, const StepArgs &st, double *tv, hipStream_t stream);
const char *inside_kernel_name(const KArgs &ka);
size_t pf_ring_lds(const KArgs &ka);
size_t outside_ring_lds(const KArgs &ka);
size_t pf_ring_scratch_floats(const KArgs &ka, int W);
const char *outside_kernel_name(const KArgs &ka);
size_t bppm_lds_bytes(const KArgs &ka, bool *gout);
size_t bppm_scratch_bytes(const KArgs &ka, int W);
hipError_t launch_bppm(const KArgs &ka, const uint8_t *seqs, int W, const int *mask, double *full, int ld,
                       double *pair_p, char *scratch, hipStream_t stream);
constexpr int NT = 512;
constexpr size_t LDS_MAX = 163840;
}  // namespace adx

using namespace adx;

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

static adx_status fail(adx_status s, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return s;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(ADX_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
    } while (0)

extern "C" const char *adx_last_error(void) { return g_err.c_str(); }
extern "C" int adx_abi_version(void) { return ADX_ABI_VERSION; }
extern "C" double adx_kT(void) { return kT_kcal(); }

// ------------------------------------------------------------------ params
struct adx_params {
    EnergyParams P;
};

extern "C" adx_status adx_params_load(const char *path, adx_params **out) {
    if (!path || !out) return fail(ADX_EINVAL, "adx_params_load: null argument");
    auto p = std::make_unique<adx_params>();
    std::string err;
    if (!load_params(path, p->P, err)) return fail(ADX_EPARAM, "%s", err.c_str());
    *out = p.release();
    return ADX_OK;
}

extern "C" void adx_params_free(adx_params *p) { delete p; }

extern "C" adx_status adx_eval_structure(const adx_params *p, const char *seq, const char *st,
                                         double *e) {
    if (!p || !seq || !st || !e) return fail(ADX_EINVAL, "adx_eval_structure: null argument");
    double v = eval_structure(p->P, seq, st);
    if (std::isnan(v)) return fail(ADX_EINVAL, "malformed structure '%s'", st);
    *e = v;
    return ADX_OK;
}

// ------------------------------------------------------------------ tables
namespace {

double boltz_d(double e_dcal) {
    if (e_dcal >= INF_E / 2) return 0.0;
    return std::exp(-e_dcal * 10.0 / kT_cal());
}
float boltz(double e_dcal) { return static_cast<float>(boltz_d(e_dcal)); }

// Loop factor of energy e (dcal/mol) spanning k scaled nucleotides: the
// Boltzmann factor exp(-e/kT) sigma^k (partition function) or the energy
// itself (MFE; INF_E and above -> MFE_BIG).  dev_types.hpp "Fold modes".
struct Fac {
    bool mfe;
    double sigma;
    float operator()(double e, int k = 0) const {
        if (mfe) return e >= INF_E ? MFE_BIG : static_cast<float>(e);
        return static_cast<float>(boltz_d(e) * std::pow(sigma, k));
    }
    float zero() const { return mfe ? MFE_BIG : 0.f; }
    float one() const { return mfe ? 0.f : 1.f; }
};

void build_tables(const EnergyParams &P, DevTables &T, bool mfe) {
    const Fac F{mfe, 1.0};
    float *flat = reinterpret_cast<float *>(&T);
    for (size_t k = 0; k < sizeof(DevTables) / sizeof(float); k++) flat[k] = F.zero();
    for (int a = 1; a <= 7; a++) {
        for (int b = 1; b <= 7; b++) T.stack[a][b] = F(P.stack[a][b]);
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) {
                T.mmH[a][x][y] = F(P.mmH[a][x][y]);
                T.mmI[a][x][y] = F(P.mmI[a][x][y]);
                T.mm1n[a][x][y] = F(P.mm1nI[a][x][y]);
                T.mm23[a][x][y] = F(P.mm23I[a][x][y]);
                T.mlstem[a][x][y] = F(ml_stem_energy(P, a, x, y));
            }
        for (int x = 0; x < 6; x++)
            for (int y = 0; y < 6; y++)
                T.ext[a][x][y] = F(ext_stem_energy(P, a, x == 5 ? -1 : x, y == 5 ? -1 : y));
        T.termAU[a] = F(a > 2 ? P.TermAU : 0);
        for (int b = 1; b <= 7; b++)
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++) {
                    T.int11[a][b][x][y] = F(P.int11[a][b][x][y]);
                    for (int z = 0; z < 5; z++) {
                        T.int21[a][b][x][y][z] = F(P.int21[a][b][x][y][z]);
                        for (int w = 0; w < 5; w++)
                            T.int22[a][b][x][y][z][w] = F(P.int22[a][b][x][y][z][w]);
                    }
                }
    }
}

struct Motif {
    std::string seq, fold;
    double energy_kcal = 0.0;
    int mode = ADX_MOTIF_AUTO;   // the per-fold facade too: RNAfold's -9.22 holo MFE
    bool present = false;
};

// Validate the ligand motif and compute its intrinsic energy (kcal/mol).
adx_status prepare_motif(const EnergyParams &P, const Motif &m, double &eint, std::vector<int> &pt) {
    const int L = static_cast<int>(m.seq.size());
    if (L < 5 || L > MAX_MOTIF || static_cast<int>(m.fold.size()) != L)
        return fail(ADX_EINVAL, "motif: sequence and fold must have equal length in [5, %d]", MAX_MOTIF);
    if (m.fold.find('&') != std::string::npos)
        return fail(ADX_EUNSUPPORTED, "motif: split (&) interior-loop motifs are not supported");
    pt.assign(L, -1);
    std::vector<int> stk;
    for (int k = 0; k < L; k++) {
        if (m.fold[k] == '(') stk.push_back(k);
        else if (m.fold[k] == ')') {
            if (stk.empty()) return fail(ADX_EINVAL, "motif: unbalanced fold '%s'", m.fold.c_str());
            pt[stk.back()] = k;
            pt[k] = stk.back();
            stk.pop_back();
        } else if (m.fold[k] != '.') {
            return fail(ADX_EINVAL, "motif: bad character in fold '%s'", m.fold.c_str());
        }
    }
    if (!stk.empty()) return fail(ADX_EINVAL, "motif: unbalanced fold '%s'", m.fold.c_str());
    if (pt[0] != L - 1)
        return fail(ADX_EUNSUPPORTED, "motif: the outermost pair must span the whole motif");
    // every pair canonical, every hairpin >= TURN, every interior loop <= MAXLOOP
    for (int k = 0; k < L; k++) {
        if (pt[k] > k) {
            if (!pair_type(base_code(m.seq[k]), base_code(m.seq[pt[k]])))
                return fail(ADX_EINVAL, "motif: non-canonical pair (%d,%d)", k, pt[k]);
            if (pt[k] - k - 1 < TURN) return fail(ADX_EINVAL, "motif: hairpin shorter than 3");
            int nb = 0, p = -1, q = -1;
            for (int t = k + 1; t < pt[k]; t++)
                if (pt[t] > t) {
                    if (++nb == 1) { p = t; q = pt[t]; }
                    t = pt[t];
                }
            if (nb == 1 && (p - k - 1) + (pt[k] - q - 1) > MAXLOOP)
                return fail(ADX_EUNSUPPORTED, "motif: interior loop larger than MAXLOOP");
        }
    }
    eint = eval_structure(P, m.seq, m.fold);
    if (std::isnan(eint)) return fail(ADX_EINVAL, "motif: cannot evaluate fold");
    return ADX_OK;
}

void build_scaled(const EnergyParams &P, double sigma, const Motif &m, double eint,
                  const std::vector<int> &mpt, DevScaled &X, bool mfe) {
    std::memset(&X, 0, sizeof X);
    const Fac F{mfe, sigma};
    auto sp = [&](int k) { return std::pow(sigma, k); };
    float *ct = X.ctab;
    // code = rtype*25 + S[q+1]*5 + S[p-1] of an inner pair; mismatchI[type2][sq1][sp1]
    for (int code = 0; code < 200; code++) {
        const int t2 = code / 25, x = (code / 5) % 5, y = code % 5;
        if (mfe) {   // energies: the inverse factor is the negated mismatch
            const int mm = t2 ? P.mmI[t2][x][y] : 0;
            ct[CT_INVMM + code] = t2 ? static_cast<float>(-mm) : MFE_BIG;
            ct[CT_BUL + code] = t2 ? static_cast<float>(-mm + (t2 > 2 ? P.TermAU : 0)) : MFE_BIG;
            ct[CT_ONEN + code] = t2 ? static_cast<float>(-mm + P.mm1nI[t2][x][y]) : MFE_BIG;
            ct[CT_M23O + code] = t2 ? static_cast<float>(P.mm23I[t2][x][y]) : MFE_BIG;
            continue;
        }
        const double mm = t2 ? boltz_d(P.mmI[t2][x][y]) : 0.0;
        const double inv = (mm > 0.0) ? 1.0 / mm : 0.0;
        ct[CT_INVMM + code] = static_cast<float>(inv);
        ct[CT_BUL + code] = static_cast<float>(inv * (t2 ? boltz_d(t2 > 2 ? P.TermAU : 0) : 0.0));
        ct[CT_ONEN + code] = static_cast<float>(inv * (t2 ? boltz_d(P.mm1nI[t2][x][y]) : 0.0));
        ct[CT_M23O + code] = static_cast<float>(t2 ? boltz_d(P.mm23I[t2][x][y]) : 0.0);
    }
    for (int a = 0; a < 8; a++)
        for (int b = 0; b < 8; b++) ct[CT_STK + a * 8 + b] = (a && b) ? F(P.stack[a][b]) : F.zero();
    for (int u = 0; u < 32; u++) {
        const int uu = std::min(u, MAXLOOP);
        ct[CT_FB + u] = F(P.bulge[uu], u + 2);
        const int nl = u;
        const double e1n = (nl >= 1 && nl + 1 <= MAXLOOP)
                               ? P.interior[nl + 1] + std::min(P.maxninio, (nl - 1) * P.ninio)
                               : INF_E;
        ct[CT_F1N + u] = F(e1n, nl + 3);
    }
    ct[CT_FSM + 0] = F(0, 2);
    ct[CT_FSM + 1] = F(P.bulge[1], 3);
    ct[CT_FSM + 2] = F(0, 4);
    ct[CT_FSM + 3] = F(0, 5);
    ct[CT_FSM + 4] = F(0, 6);
    ct[CT_FSM + 5] = F(P.interior[5] + P.ninio, 7);
    ct[CT_FSM + 6] = F(P.TermAU);
    ct[CT_ONE] = F.one();
    for (int u = 6; u <= MAXLOOP; u++)
        for (int n1 = 2; n1 < 2 + FG_ROW; n1++) {
            const int n2 = u - n1;
            X.fgen[(u - 6) * FG_ROW + n1 - 2] =
                n2 >= 2 ? F(P.interior[u] + std::min(P.maxninio, std::abs(n1 - n2) * P.ninio), u + 2) : F.zero();
        }
    for (int k = 0; k < 32; k++) {
        X.il[k] = (mfe && k <= MAXLOOP) ? static_cast<float>(P.interior[k]) : 0.f;
        X.nin[k] = mfe ? static_cast<float>(std::min(P.maxninio, k * P.ninio)) : 0.f;
    }
    // term lists ordered by u (dev_types.hpp NS_MAX)
    int ns = 0, ng = 0;
    auto addS = [&](int kind, int n1, int n2, float f) {
        X.s_kind[ns] = static_cast<uint8_t>(kind);
        X.s_n1[ns] = static_cast<uint8_t>(n1);
        X.s_n2[ns] = static_cast<uint8_t>(n2);
        X.s_f[ns] = f;
        ns++;
    };
    for (int u = 0; u <= MAXLOOP; u++) {
        if (u == 0) addS(TK_STK, 0, 0, ct[CT_FSM + 0]);
        if (u == 1) { addS(TK_B1, 0, 1, ct[CT_FSM + 1]); addS(TK_B1, 1, 0, ct[CT_FSM + 1]); }
        if (u == 2) addS(TK_I11, 1, 1, ct[CT_FSM + 2]);
        if (u == 3) { addS(TK_I12, 1, 2, ct[CT_FSM + 3]); addS(TK_I21, 2, 1, ct[CT_FSM + 3]); }
        if (u == 4) addS(TK_I22, 2, 2, ct[CT_FSM + 4]);
        if (u == 5) { addS(TK_M23, 2, 3, ct[CT_FSM + 5]); addS(TK_M23, 3, 2, ct[CT_FSM + 5]); }
        if (u >= 2) { addS(TK_BUL, 0, u, ct[CT_FB + u]); addS(TK_BUL, u, 0, ct[CT_FB + u]); }
        if (u >= 4) { addS(TK_1N, 1, u - 1, ct[CT_F1N + u - 1]); addS(TK_1N, u - 1, 1, ct[CT_F1N + u - 1]); }
        for (int n1 = 2; u >= 6 && n1 <= u - 2; n1++) {
            X.g_n1[ng] = static_cast<uint8_t>(n1);
            X.g_u[ng] = static_cast<uint8_t>(u);
            X.g_f[ng] = X.fgen[(u - 6) * FG_ROW + n1 - 2];
            ng++;
        }
        X.s_cnt[u] = ns;
        X.g_cnt[u] = ng;
    }
    X.s_cnt[31] = ns;
    X.g_cnt[31] = ng;
    for (int k = 0; k < NMAX + 4; k++) X.sig[k] = F(0, k);
    for (int u = 0; u <= NMAX; u++) {
        if (mfe) {   // the MFE truncates the long-loop extrapolation to dcal (oracle E_hairpin_int)
            const int e = (u <= 30) ? P.hairpin[u] : P.hairpin[30] + static_cast<int>(P.lxc * std::log(u / 30.0));
            X.hp[u] = F(e);
        } else {
            const double e = (u <= 30) ? P.hairpin[u] : P.hairpin[30] + P.lxc * std::log(u / 30.0);
            X.hp[u] = F(e, u + 2);
        }
    }
    const double mlb = boltz_d(P.MLbase);
    for (int t = 0; t <= NMAX; t++)
        X.pwml[t] = mfe ? static_cast<float>(t * P.MLbase) : static_cast<float>(std::pow(mlb * sigma, t));
    X.mlclosing = F(P.MLclosing, 2);
    X.mlbase_sig = F(P.MLbase, 1);
    int nsp = 0;
    auto add_special = [&](const std::vector<std::pair<std::string, int>> &tab) {
        for (auto &e : tab) {
            if (nsp >= MAX_SPECIAL_HP) break;
            std::vector<uint8_t> codes(e.first.size());
            for (size_t k = 0; k < e.first.size(); k++) codes[k] = static_cast<uint8_t>(base_code(e.first[k]));
            X.sp_key[nsp] = hp_key(codes.data(), 0, static_cast<int>(codes.size()));
            X.sp_val[nsp] = F(e.second, static_cast<int>(codes.size()));
            nsp++;
        }
    };
    add_special(P.triloops);
    add_special(P.tetraloops);
    add_special(P.hexaloops);
    X.n_special = nsp;
    X.log_sigma = mfe ? 0.0 : std::log(sigma);
    X.kT = kT_kcal();
    if (m.present) {
        const int L = static_cast<int>(m.seq.size());
        X.motif_len = L;
        for (int k = 0; k < L; k++) {
            X.motif_code[k] = static_cast<uint8_t>(base_code(m.seq[k]));
            X.motif_pt[k] = static_cast<int8_t>(mpt[k]);
        }
        const bool replace = m.mode == ADX_MOTIF_REPLACE || (m.mode == ADX_MOTIF_AUTO && mfe);
        const double beff = replace ? m.energy_kcal - eint : m.energy_kcal;
        if (mfe) {   // min-plus image of the extra term: the formed motif's energy, rounded once to dcal
            X.motif_extra = static_cast<float>(std::lround(100.0 * (eint + beff)));
        } else {
            const double extra = boltz_d(eint * 100.0) * (boltz_d(beff * 100.0) - 1.0) * sp(L);
            X.motif_extra = static_cast<float>(extra);
        }
    }
}

// Dot-bracket hard constraint (DB_DEFAULT | ENFORCE_BP, scoring.cc:61-62) ->
// five byte arrays of length N+2: up, dn, ptn, enc, flg (see kernels.hip).
adx_status build_constraint(const std::string &cst, int N, std::vector<uint8_t> &out) {
    const int np = N + 2;
    out.assign(5 * np, 0);
    std::vector<int> partner(np, 0), enc(np, 0), unp(np, 1), flg(np, 0), stk;
    for (int i = 1; i <= N; i++) {
        const char c = cst.empty() ? '.' : cst[i - 1];
        enc[i] = stk.empty() ? 0 : stk.back();
        if (c == '(') stk.push_back(i);
        else if (c == ')') {
            if (stk.empty()) return fail(ADX_ECONSTRAINT, "unbalanced ')' in constraint '%s'", cst.c_str());
            int a = stk.back();
            stk.pop_back();
            partner[a] = i;
            partner[i] = a;
            enc[i] = stk.empty() ? 0 : stk.back();
        }
    }
    if (!stk.empty()) return fail(ADX_ECONSTRAINT, "unbalanced '(' in constraint '%s'", cst.c_str());
    for (int i = 1; i <= N; i++) {
        const char c = cst.empty() ? '.' : cst[i - 1];
        if (c == 'x') flg[i] |= 1;
        if (c == '<') flg[i] |= 2;
        if (c == '>') flg[i] |= 4;
        if (c == '|' || c == '<' || c == '>' || partner[i]) unp[i] = 0;
    }
    std::vector<int> up(np + 1, 0), dn(np, 0);
    for (int i = N; i >= 1; i--) up[i] = unp[i] ? up[i + 1] + 1 : 0;
    for (int i = 1; i <= N; i++) dn[i] = unp[i] ? dn[i - 1] + 1 : 0;
    for (int k = 0; k < np; k++) {
        out[k] = static_cast<uint8_t>(std::min(up[k], 255));
        out[np + k] = static_cast<uint8_t>(std::min(dn[k], 255));
        out[2 * np + k] = static_cast<uint8_t>(partner[k]);
        out[3 * np + k] = static_cast<uint8_t>(enc[k]);
        out[4 * np + k] = static_cast<uint8_t>(flg[k]);
    }
    return ADX_OK;
}

std::vector<uint8_t> encode(const std::string &s) {
    std::vector<uint8_t> v(s.size());
    for (size_t k = 0; k < s.size(); k++) v[k] = static_cast<uint8_t>(base_code(s[k]));
    return v;
}

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    ~DevBuf() { reset(); }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        reset();
        n = count;
        return hipMalloc(reinterpret_cast<void **>(&p), std::max<size_t>(count, 1) * sizeof(T));
    }
    hipError_t upload(const T *src, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess) return e;
        return hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

// One folding problem: energy tables, scaled constants, variants,
// constraint blobs and score-term map on one device.
struct Problem {
    int device = 0;
    hipStream_t stream = nullptr;
    const EnergyParams *P = nullptr;
    int Nraw = 0, Nmax = 0;
    Motif motif;
    double motif_eint = 0.0;
    std::vector<int> motif_pt;
    double g0 = -0.30;  // assumed free energy per nucleotide for the pf scale
    std::vector<DevVariant> variants;
    std::vector<int> vmac;       // per variant: macrostate index, -1 = unconstrained
    std::vector<int> groups2;    // variant pairs folded in lockstep (kernels.hip pf_group)
    std::vector<uint8_t> cons;
    std::vector<uint8_t> ctx_seq;
    std::vector<int> ctx_off;
    std::vector<DevTermMap> tmap;
    int n_terms = 0, n_ctx_eff = 1;
    bool qbm = true;
    int mode = 0;                // 0 = partition functions, 1 = MFE (ADX_FOLD_*)
    DevBuf<DevTables> dT;
    DevBuf<DevScaled> dX;
    DevBuf<DevVariant> dV;
    DevBuf<uint8_t> dCons, dCtxSeq;
    DevBuf<int> dCtxOff;
    DevBuf<DevTermMap> dTmap;
    DevBuf<int> dGroups2;
    // base-pair probability terms: outside variants, requested pairs, per-walker results
    std::vector<int> bvars;
    std::vector<int> pairs;      // [n][3]: bvars index, i, j (1-based folded coordinates)
    DevBuf<int> dBvars, dPairs, dBvarSlot;
    DevBuf<double> dPairP;
    DevBuf<char> dScratch;       // outside tables in HBM when they do not fit LDS
    bool pf_ring = false;        // PF folds by pf_ring_kernel (fixes the slot layout, kernels.hip)
    DevBuf<float> dRingScr;      // its qb scratch for stateless launches
    // MFE: packed 16-bit copies of the energy tables (kernels.hip MinPlus16)
    DevBuf<DevTables> dT16;
    DevBuf<DevScaled> dX16;
    DevBuf<int> dOvf;
    bool mfe16 = false;
    bool mfe_cells_ok = false;   // Ninio saturated from |n1-n2| = 5 on, MLbase >= 0 (mfe_cells.hip)
    // incremental-fold state of the MC walkers (kernels.hip Inc)
    DevBuf<float> dTab;
    DevBuf<float> dGstep;        // [W][n_variants] energies of the step's folds (pf_cells_kernel,
                                 //   and the pair-term score that waits for the outside pass)
    DevBuf<uint8_t> dCur, dValid;
    DevBuf<int> dChg;
    DevBuf<int> dOrder;          // launch order of a rescore's folds (KArgs::order, order_kernel)
    DevBuf<uint8_t> dCls;        // the folds' weight classes (KArgs::ocls, the proposals' or a rescore's)
    size_t tab_slot = 0;
    bool state_on = false;   // set for MC launches only (not for adx_score_batch)
    std::unique_ptr<DevTables> hT;
    std::unique_ptr<DevScaled> hX;

    ~Problem() {
        if (stream) (void)hipStreamDestroy(stream);
    }

    double sigma() const { return std::exp(g0 / kT_kcal()); }

    adx_status init_device() {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            return fail(ADX_ENODEV, "no HIP device visible (the engine requires a gfx950 GPU)");
        if (device < 0 || device >= ndev) return fail(ADX_ENODEV, "device %d not present (%d visible)", device, ndev);
        HIP_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(ADX_ENODEV, "device %d is %s, the kernels are built for gfx950", device, prop.gcnArchName);
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        return ADX_OK;
    }

    KArgs kargs() const {
        KArgs ka{};
        ka.T = dT.p;
        ka.X = dX.p;
        ka.variants = dV.p;
        ka.cons = dCons.p;
        ka.ctx_seq = dCtxSeq.p;
        ka.ctx_off = dCtxOff.p;
        ka.tmap = dTmap.p;
        ka.n_variants = static_cast<int>(variants.size());
        ka.n_terms = n_terms;
        ka.n_ctx_eff = n_ctx_eff;
        ka.Nraw = Nraw;
        ka.Nmax = Nmax;
        ka.cells = Nmax >= 5 ? (Nmax - 4) * (Nmax - 3) / 2 : 1;
        ka.groups2 = dGroups2.p;
        ka.n_groups2 = static_cast<int>(groups2.size() / 2);
        ka.opt = 0;
        ka.mode = mode;
        ka.bvars = dBvars.p;
        ka.n_bvars = static_cast<int>(bvars.size());
        ka.bvar_slot = dBvarSlot.p;
        ka.pairs = dPairs.p;
        ka.n_pairs = static_cast<int>(pairs.size() / 3);
        ka.pair_p = dPairP.p;
        ka.bppm_scratch = dScratch.p;
        ka.T16 = mfe16 ? dT16.p : nullptr;
        ka.X16 = mfe16 ? dX16.p : nullptr;
        ka.ovf = mfe16 ? dOvf.p : nullptr;
        ka.mfe_cells_ok = mfe16 && mfe_cells_ok ? 1 : 0;
        const bool st = state_on && dTab.p && !std::getenv("ADX_NO_INCR");
        ka.tab = st ? dTab.p : nullptr;
        ka.tab_slot = tab_slot;
        ka.cur_slot = st ? dCur.p : nullptr;
        ka.tab_valid = st ? dValid.p : nullptr;
        ka.chg = st ? dChg.p : nullptr;
        ka.order = st && !std::getenv("ADX_NO_ORDER") ? dOrder.p : nullptr;
        ka.ocls = dCls.p;
        ka.gstep = dGstep.p;
        ka.pf_ring = pf_ring ? 1 : 0;
        ka.ring_scratch = dRingScr.p;
        return ka;
    }

    adx_status choose_layout() {
        KArgs ka = kargs();
        const char *env = std::getenv("ADX_QBM");
        const size_t with = lds_bytes(ka, true, NT), without = lds_bytes(ka, false, NT);
        if (env) qbm = std::atoi(env) != 0;
        else if (with * 2 <= LDS_MAX) qbm = true;
        else if (without * 2 <= LDS_MAX) qbm = false;
        else qbm = with <= LDS_MAX;
        if (lds_bytes(ka, qbm, NT) > LDS_MAX)
            return fail(ADX_EUNSUPPORTED, "sequence length %d needs %zu B of LDS (> %zu)", Nmax,
                        lds_bytes(ka, qbm, NT), LDS_MAX);
        return ADX_OK;
    }

    adx_status upload_scaled() {
        build_scaled(*P, sigma(), motif, motif_eint, motif_pt, *hX, mode == 1);
        HIP_TRY(dX.upload(hX.get(), 1, stream));
        return ADX_OK;
    }

    // MFE: the energy tables as packed int16 pairs (value duplicated in both
    // halves; >= MFE_BIG/2 -> 0x7FFF).  Returns false when a value does not fit.
    static bool pack16(float *a, size_t n) {
        for (size_t k = 0; k < n; k++) {
            const double e = a[k];
            uint32_t h;
            if (e >= 0.5 * MFE_BIG) h = 0x7FFFu;
            else if (e <= -16384.0 || e >= 16384.0 || e != std::floor(e)) return false;
            else h = static_cast<uint16_t>(static_cast<int16_t>(e));
            const uint32_t w = h | (h << 16);
            std::memcpy(&a[k], &w, 4);
        }
        return true;
    }
    adx_status upload_mfe16() {
        mfe16 = false;
        if (mode != 1 || std::getenv("ADX_NO_MFE16")) return ADX_OK;
        auto T16 = std::make_unique<DevTables>(*hT);
        auto X16 = std::make_unique<DevScaled>(*hX);
        bool ok = pack16(reinterpret_cast<float *>(T16.get()), sizeof(DevTables) / sizeof(float));
        ok = ok && pack16(X16->ctab, CT_SIZE) && pack16(X16->fgen, FG_SIZE) && pack16(X16->il, 32) && pack16(X16->nin, 32) && pack16(X16->s_f, NS_MAX) &&
             pack16(X16->g_f, NG_MAX) && pack16(X16->sig, NMAX + 4) && pack16(X16->hp, NMAX + 1) &&
             pack16(X16->pwml, NMAX + 1) && pack16(&X16->mlclosing, 1) && pack16(&X16->mlbase_sig, 1) &&
             pack16(X16->sp_val, MAX_SPECIAL_HP) && pack16(&X16->motif_extra, 1);
        if (!ok) return ADX_OK;   // FP32 MinPlus only
        {   // mfe_cells.hip interior-loop records (both halves non-negative: a plain 32-bit add)
            uint32_t il[32], nin[32], ct[CT_SIZE];
            std::memcpy(il, X16->il, sizeof il);
            std::memcpy(nin, X16->nin, sizeof nin);
            std::memcpy(ct, X16->ctab, sizeof ct);
            for (int u = 0; u < 32; u++)
                for (int f = 0; f < 8; f++)
                    X16->ku16[u][f] = f < 6 ? ((u >= 6 && u <= 30) ? il[u] + nin[f] : 0u)
                                    : f == 6 ? ct[CT_FB + u] : (u >= 1 ? ct[CT_F1N + u - 1] : 0x7FFF7FFFu);
        }
        HIP_TRY(dT16.upload(T16.get(), 1, stream));
        HIP_TRY(dX16.upload(X16.get(), 1, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        mfe16 = true;
        mfe_cells_ok = P->MLbase >= 0;
        for (int k = 5; k <= MAXLOOP; k++)
            if (std::min(P->maxninio, k * P->ninio) != std::min(P->maxninio, 5 * P->ninio)) mfe_cells_ok = false;
        return ADX_OK;
    }
    // per walker two slots of every group's tables: sized for the largest kernel
    // configuration (P = 2 value arrays, one group per variant)
    adx_status alloc_state(int W) {
        tab_slot = size_t(variants.size()) * inc_group_floats(kargs().cells, Nmax, 2);
        // the MFE16 slots' per-cell codes follow the groups' tables (dev_types.hpp)
        const int ng = int((variants.size() + 1) / 2) + int(variants.size());
        tab_slot = std::max(tab_slot, inc_cc_offset(kargs().cells, Nmax, ng, ng));
        tab_slot = std::max(tab_slot, inc_cc_offset_pf(kargs().cells, Nmax, ng, ng));
        tab_slot = (tab_slot + 3) / 4 * 4;   // 16-byte aligned slots (the codes are read as uint4)
        HIP_TRY(dTab.alloc(size_t(W) * 2 * tab_slot));
        HIP_TRY(dCur.alloc(W));
        HIP_TRY(dValid.alloc(W));
        HIP_TRY(dChg.alloc(size_t(W) * 2));
        HIP_TRY(dOrder.alloc(W));
        HIP_TRY(dCls.alloc(W));
        HIP_TRY(hipMemsetAsync(dCls.p, 64, W, stream));   // "not scored" until a proposal or rescore sets it
        if (adx_status sg = ensure_gstep(W)) return sg;
        HIP_TRY(hipMemsetAsync(dCur.p, 1, W, stream));     // the initial fold writes slot 0
        HIP_TRY(hipMemsetAsync(dValid.p, 0, W, stream));
        HIP_TRY(hipMemsetAsync(dChg.p, 0xff, sizeof(int) * 2 * W, stream));
        return ADX_OK;
    }
    adx_status ensure_ovf(int W) {
        if (mfe16 && dOvf.n < size_t(W)) {
            HIP_TRY(dOvf.alloc(W));
            HIP_TRY(hipMemsetAsync(dOvf.p, 0, sizeof(int) * W, stream));
        }
        return ADX_OK;
    }

    adx_status upload_all() {
        hT = std::make_unique<DevTables>();
        hX = std::make_unique<DevScaled>();
        build_tables(*P, *hT, mode == 1);
        HIP_TRY(dT.upload(hT.get(), 1, stream));
        adx_status s = upload_scaled();
        if (s) return s;
        HIP_TRY(dV.upload(variants.data(), variants.size(), stream));
        HIP_TRY(dCons.upload(cons.data(), cons.size(), stream));
        HIP_TRY(dCtxSeq.upload(ctx_seq.data(), ctx_seq.size(), stream));
        HIP_TRY(dCtxOff.upload(ctx_off.data(), ctx_off.size(), stream));
        HIP_TRY(dTmap.upload(tmap.data(), tmap.size(), stream));
        // apo / holo variants of one (context, macrostate) share every cell: pair them
        groups2.clear();
        if (vmac.size() != variants.size()) vmac.assign(variants.size(), -1);
        std::vector<char> used(variants.size(), 0);
        for (size_t v = 0; v < variants.size(); v++) {
            if (used[v]) continue;
            used[v] = 1;
            size_t mate = v;
            for (size_t w = v + 1; w < variants.size(); w++) {
                if (!used[w] && variants[w].ctx == variants[v].ctx && vmac[w] == vmac[v] &&
                    variants[w].N == variants[v].N && variants[w].motif != variants[v].motif) {
                    mate = w;
                    used[w] = 1;
                    break;
                }
            }
            groups2.push_back(static_cast<int>(v));
            groups2.push_back(static_cast<int>(mate));
        }
        HIP_TRY(dGroups2.upload(groups2.data(), groups2.size(), stream));
        HIP_TRY(dBvars.upload(bvars.data(), bvars.size(), stream));
        // every outside variant's position in the groups2 slot layout (the outside
        // kernels read the proposal's inside tables there): an invariant, not a search
        std::vector<int> bslot(bvars.size(), -1);
        for (size_t b = 0; b < bvars.size(); b++)
            for (size_t g = 0; g < groups2.size() && bslot[b] < 0; g++)
                if (groups2[g] == bvars[b]) bslot[b] = static_cast<int>(g);
        for (size_t b = 0; b < bslot.size(); b++)
            if (bslot[b] < 0) return fail(ADX_EINVAL, "internal: outside variant %d has no fold group", bvars[b]);
        HIP_TRY(dBvarSlot.upload(bslot.data(), bslot.size(), stream));
        HIP_TRY(dPairs.upload(pairs.data(), pairs.size(), stream));
        HIP_TRY(hipStreamSynchronize(stream));
        // PF folds longer than pf_cells covers take the ring kernel (pf_ring.hip).
        // One choice per context: it fixes the layout of the walkers' stored
        // tables, which every later kernel of the context must read the same way.
        {
            pf_ring = false;
            const char *e = std::getenv("ADX_PF_KERNEL");
            const bool rows = e && std::strcmp(e, "rows") == 0;
            const KArgs k = kargs();
            pf_ring = mode == 0 && !rows && pf_ring_lds(k) > 0 && (pairs.empty() || outside_ring_lds(k) > 0);
        }
        s = upload_mfe16();
        if (s) return s;
        if (!pairs.empty() && bppm_lds_bytes(kargs(), nullptr) == 0)
            return fail(ADX_EUNSUPPORTED, "base-pair probabilities of length %d do not fit one CU's LDS yet", Nmax);
        return choose_layout();
    }

    // per-walker pair-probability buffer (grow-only)
    adx_status ensure_pairs(int W) {
        const size_t need = size_t(W) * (pairs.size() / 3);
        if (need > 0 && dPairP.n < need) HIP_TRY(dPairP.alloc(need));
        return ensure_scratch(kargs(), W);
    }
    adx_status ensure_scratch(const KArgs &ka, int W) {
        const size_t need = bppm_scratch_bytes(ka, W);
        if (need > 0 && dScratch.n < need) HIP_TRY(dScratch.alloc(need));
        return ADX_OK;
    }

    adx_status ensure_gstep(int W) {
        const size_t need = size_t(W) * variants.size();
        if (dGstep.n < need) HIP_TRY(dGstep.alloc(need));
        return ADX_OK;
    }

    // the per-walker buffers a fold of W walkers writes (grow-only)
    adx_status prepare(int W) {
        adx_status so = ensure_ovf(W);
        if (so) return so;
        so = ensure_gstep(W);
        if (so) return so;
        if (pf_ring) {   // qb scratch of the stateless ring folds
            const size_t need = pf_ring_scratch_floats(kargs(), W);
            if (dRingScr.n < need) HIP_TRY(dRingScr.alloc(need));
        }
        return pairs.empty() ? ADX_OK : ensure_pairs(W);
    }

    // Score W sequences (device pointer of W*Nraw codes); outputs are device pointers.
    adx_status score(const uint8_t *dseqs, int W, double *dscores, double *dterms, float *ddG) {
        adx_status so = prepare(W);
        if (so) return so;
        if (!pairs.empty())
            HIP_TRY(launch_bppm(kargs(), dseqs, W, nullptr, nullptr, 0, dPairP.p, dScratch.p, stream));
        HIP_TRY(launch_score(kargs(), qbm, dseqs, W, dscores, dterms, ddG, stream));
        return ADX_OK;
    }
};

// pick a pf scale from the ensemble energy of a reference sequence
adx_status calibrate(Problem &pb, const std::vector<uint8_t> &codes) {
    DevBuf<uint8_t> dseq;
    DevBuf<double> dsc;
    DevBuf<float> ddg;
    HIP_TRY(dseq.upload(codes.data(), codes.size(), pb.stream));
    HIP_TRY(dsc.alloc(1));
    HIP_TRY(ddg.alloc(pb.variants.size()));
    std::vector<float> g(pb.variants.size());
    for (int attempt = 0; attempt < 6; attempt++) {
        adx_status s = pb.upload_scaled();
        if (s) return s;
        s = pb.score(dseq.p, 1, dsc.p, nullptr, ddg.p);
        if (s) return s;
        HIP_TRY(hipMemcpyAsync(g.data(), ddg.p, g.size() * sizeof(float), hipMemcpyDeviceToHost, pb.stream));
        HIP_TRY(hipStreamSynchronize(pb.stream));
        // variant 0 is always the unconstrained apo ensemble of the first context
        const double G = g[0];
        const int N = pb.variants[0].N;
        if (std::isfinite(G) && N > 0) {
            const double g_new = std::min(-0.05, G / N);
            if (std::fabs(g_new - pb.g0) < 1e-9) return ADX_OK;
            pb.g0 = g_new;
            return pb.upload_scaled();
        }
        pb.g0 *= 2.0;  // overflow: scale harder and retry
    }
    return fail(ADX_EINVAL, "could not find a partition-function scale for this sequence");
}

}  // namespace

// ================================================================== fold layer
struct adx_fold {
    const adx_params *params = nullptr;
    std::string seq;
    int with_bppm = 0;
    int device = 0;
    std::string constraint;  // accumulated (last one wins, like a fresh DB constraint)
    Motif motif;
    std::vector<double> bpp; // cached N*N probabilities (scoring.cc:41-44 computes them once)
};

extern "C" adx_status adx_fold_create(const adx_params *p, const char *seq, int with_bppm, int device,
                                      adx_fold **out) {
    if (!p || !seq || !out) return fail(ADX_EINVAL, "adx_fold_create: null argument");
    const int N = static_cast<int>(std::strlen(seq));
    if (N < 1 || N > NMAX) return fail(ADX_EINVAL, "sequence length %d outside [1, %d]", N, NMAX);
    auto f = std::make_unique<adx_fold>();
    f->params = p;
    f->seq = seq;
    for (auto &c : f->seq) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
    f->with_bppm = with_bppm;
    f->device = device;
    *out = f.release();
    return ADX_OK;
}

extern "C" adx_status adx_fold_add_motif(adx_fold *f, const char *mseq, const char *mfold, double e) {
    if (!f || !mseq || !mfold) return fail(ADX_EINVAL, "adx_fold_add_motif: null argument");
    f->motif.seq = mseq;
    for (auto &c : f->motif.seq) c = static_cast<char>(std::toupper(static_cast<unsigned char>(c)));
    f->motif.fold = mfold;
    f->motif.energy_kcal = e;
    f->motif.present = true;
    f->bpp.clear();
    return ADX_OK;
}

extern "C" adx_status adx_fold_add_constraint(adx_fold *f, const char *db) {
    if (!f || !db) return fail(ADX_EINVAL, "adx_fold_add_constraint: null argument");
    if (std::strlen(db) != f->seq.size())
        return fail(ADX_ECONSTRAINT, "constraint length %zu != sequence length %zu", std::strlen(db), f->seq.size());
    std::vector<uint8_t> tmp;
    adx_status s = build_constraint(db, static_cast<int>(f->seq.size()), tmp);
    if (s) return s;
    f->constraint = db;
    f->bpp.clear();
    return ADX_OK;
}

// One fold of the compound f in mode 0 (partition function) or 1 (MFE).
static adx_status fold_energy(adx_fold *f, int mode, float *energy, std::vector<double> *bpp = nullptr) {
    Problem pb;
    pb.mode = mode;
    pb.device = f->device;
    pb.P = &f->params->P;
    adx_status s = pb.init_device();
    if (s) return s;
    const int N = static_cast<int>(f->seq.size());
    pb.Nraw = pb.Nmax = N;
    pb.motif = f->motif;
    if (pb.motif.present) {
        s = prepare_motif(*pb.P, pb.motif, pb.motif_eint, pb.motif_pt);
        if (s) return s;
    }
    // variant 0: the ensemble this fold compound currently describes
    std::vector<uint8_t> c;
    s = build_constraint(f->constraint, N, c);
    if (s) return s;
    pb.cons = c;
    pb.variants.push_back(DevVariant{N, 0, -1, 0, pb.motif.present ? 1 : 0, 0});
    pb.ctx_seq.assign(1, 0);
    pb.ctx_off.assign(4, 0);
    pb.tmap.assign(1, DevTermMap{0, 0, 1, 0.0});
    pb.n_terms = 0;
    s = pb.upload_all();
    if (s) return s;
    std::vector<uint8_t> codes = encode(f->seq);
    DevBuf<uint8_t> dseq;
    DevBuf<double> dsc;
    DevBuf<float> ddg;
    HIP_TRY(dseq.upload(codes.data(), codes.size(), pb.stream));
    HIP_TRY(dsc.alloc(1));
    HIP_TRY(ddg.alloc(1));
    float g = NAN;
    if (mode == 1) {   // integer min-plus: no scale to calibrate
        s = pb.score(dseq.p, 1, dsc.p, nullptr, ddg.p);
        if (s) return s;
        HIP_TRY(hipMemcpyAsync(&g, ddg.p, sizeof(float), hipMemcpyDeviceToHost, pb.stream));
        HIP_TRY(hipStreamSynchronize(pb.stream));
        *energy = g;
        return ADX_OK;
    }
    for (int attempt = 0; attempt < 6; attempt++) {
        s = pb.score(dseq.p, 1, dsc.p, nullptr, ddg.p);
        if (s) return s;
        HIP_TRY(hipMemcpyAsync(&g, ddg.p, sizeof(float), hipMemcpyDeviceToHost, pb.stream));
        HIP_TRY(hipStreamSynchronize(pb.stream));
        if (std::isfinite(g) || (std::isinf(g) && g > 0)) {
            // +inf = empty (constrained) ensemble; recalibrate once for accuracy
            if (attempt == 0 && std::isfinite(g) && N > 0) {
                pb.g0 = std::min(-0.05, static_cast<double>(g) / N);
                s = pb.upload_scaled();
                if (s) return s;
                continue;
            }
            break;
        }
        pb.g0 *= 2.0;
        s = pb.upload_scaled();
        if (s) return s;
    }
    *energy = g;
    if (bpp) {   // outside pass on the calibrated scale
        bpp->assign(size_t(N) * N, 0.0);
        if (!std::isfinite(g)) return ADX_OK;   // empty ensemble: every probability is 0
        pb.bvars.assign(1, 0);
        HIP_TRY(pb.dBvars.upload(pb.bvars.data(), 1, pb.stream));
        if (bppm_lds_bytes(pb.kargs(), nullptr) == 0)
            return fail(ADX_EUNSUPPORTED, "base-pair probabilities of length %d do not fit one CU's LDS yet", N);
        s = pb.ensure_scratch(pb.kargs(), 1);
        if (s) return s;
        const KArgs ka = pb.kargs();
        DevBuf<double> dfull;
        HIP_TRY(dfull.alloc(size_t(N) * N));
        HIP_TRY(hipMemsetAsync(dfull.p, 0, sizeof(double) * N * N, pb.stream));
        HIP_TRY(launch_bppm(ka, dseq.p, 1, nullptr, dfull.p, N, nullptr, ka.bppm_scratch, pb.stream));
        HIP_TRY(hipMemcpyAsync(bpp->data(), dfull.p, sizeof(double) * N * N, hipMemcpyDeviceToHost, pb.stream));
        HIP_TRY(hipStreamSynchronize(pb.stream));
    }
    return ADX_OK;
}

extern "C" adx_status adx_fold_pf(adx_fold *f, float *energy) {
    if (!f || !energy) return fail(ADX_EINVAL, "adx_fold_pf: null argument");
    return fold_energy(f, 0, energy);
}

extern "C" adx_status adx_fold_mfe(adx_fold *f, float *energy) {
    if (!f || !energy) return fail(ADX_EINVAL, "adx_fold_mfe: null argument");
    return fold_energy(f, 1, energy);
}

extern "C" adx_status adx_fold_bpp(adx_fold *f, int i, int j, double *prob) {
    if (!f || !prob) return fail(ADX_EINVAL, "adx_fold_bpp: null argument");
    const int N = static_cast<int>(f->seq.size());
    if (i < 1 || j < 1 || i > N || j > N) return fail(ADX_EINVAL, "adx_fold_bpp: (%d, %d) outside [1, %d]", i, j, N);
    if (f->bpp.empty()) {
        float g = 0.f;
        adx_status s = fold_energy(f, 0, &g, &f->bpp);
        if (s) {
            f->bpp.clear();
            return s;
        }
    }
    *prob = (i != j) ? f->bpp[size_t(i - 1) * N + (j - 1)] : 0.0;
    return ADX_OK;
}

extern "C" void adx_fold_free(adx_fold *f) { delete f; }

// ================================================================== MC layer
struct adx_ctx {
    Problem pb;
    std::string templ;
    std::vector<std::string> macrostates;
    std::vector<adx_term> terms;
    adx_thermostat thermo{};
    int n_contexts = 0;
    std::vector<int> mut;
    std::vector<int> clo_off, clo_pos, clo_err;
    std::vector<uint8_t> clo_par;
    std::vector<std::string> clo_msg;
    // walker state
    int W = 0;
    long long step = 0;
    DevBuf<uint8_t> cur_seq;
    DevBuf<double> cur_score, last_diff, auto_T, train;
    DevBuf<uint32_t> mtA, mtC;
    DevBuf<int64_t> counters;
    DevBuf<int> ntrain, err;
    DevBuf<uint8_t> prop_seq;
    DevBuf<double> prop_score, temp, u;
    DevBuf<int> changed, pick, bcode;
    DevBuf<int> d_mut, d_clo_off, d_clo_pos, d_clo_err;
    DevBuf<uint8_t> d_clo_par;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0.0;
    std::string inside_kernel, outside_kernel;   // what the last adx_run_steps launched
    double score_ms_total = 0.0;   // sum of the score-kernel launch durations of the last run
    double inside_ms_total = 0.0, outside_ms_total = 0.0;   // the same windows split (inside, outside)
    int score_launches = 0;

    ~adx_ctx() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
    }
};

namespace {

const char *move_error_text(int code) {
    switch (code) {
    case 1: return "mismatched base-pair in macrostate";
    case 2: return "position can be mutated, but it's base-paired to a position which can't be";
    case 3: return "no way to satisfy all base pairing constraints.";
    default: return "unknown move error";
    }
}

// mutate_recursively (sampling.cc:195-282) on the template, recording the
// closure of `pos` with its base parity and the first error the reference
// would throw.  The result does not depend on the base chosen.
int closure(const std::string &seq, const std::vector<std::string> &ms, int pos,
            std::vector<std::pair<int, int>> &out) {
    const int n = static_cast<int>(seq.size());
    std::vector<int> par(n, -1);
    // recursive DFS in the reference's order
    std::function<int(int, int)> rec = [&](int p, int parity) -> int {
        par[p] = parity;
        out.push_back({p, parity});
        for (const auto &mac : ms) {
            char open, close;
            int stepv;
            if (mac[p] == '(') { open = '('; close = ')'; stepv = 1; }
            else if (mac[p] == ')') { open = ')'; close = '('; stepv = -1; }
            else continue;
            int level = 1, partner = p;
            while (level != 0) {
                partner += stepv;
                if (partner < 0 || partner >= n) return 1;
                level += (mac[partner] == open);
                level -= (mac[partner] == close);
            }
            if (!std::isupper(static_cast<unsigned char>(seq[partner]))) return 2;
            if (par[partner] < 0) {
                int rc = rec(partner, parity ^ 1);
                if (rc) return rc;
            } else if (par[partner] != (parity ^ 1)) {
                return 3;
            }
        }
        return 0;
    };
    return rec(pos, 0);
}

}  // namespace

extern "C" adx_status adx_ctx_create(const adx_run_desc *d, adx_ctx **out) {
    if (!d || !out || !d->params || !d->sequence) return fail(ADX_EINVAL, "adx_ctx_create: null argument");
    auto c = std::make_unique<adx_ctx>();
    Problem &pb = c->pb;
    pb.device = d->device;
    pb.P = &d->params->P;
    c->templ = d->sequence;
    const int N = static_cast<int>(c->templ.size());
    if (N < 1) return fail(ADX_EINVAL, "empty sequence");
    for (int m = 0; m < d->n_macrostates; m++) {
        std::string s = d->macrostates[m];
        if (static_cast<int>(s.size()) != N)
            return fail(ADX_EINVAL, "constraint length doesn't match sequence length");
        c->macrostates.push_back(s);
    }
    if (d->n_terms < 0 || d->n_terms > MAX_TERMS) return fail(ADX_EINVAL, "n_terms out of range");
    for (int t = 0; t < d->n_terms; t++) {
        const adx_term &T = d->terms[t];
        if (T.kind == ADX_TERM_PAIR) {
            if (T.pair_i < 0 || T.pair_j >= N || T.pair_j - T.pair_i < 1)
                return fail(ADX_EINVAL, "term %d: pair (%d, %d) outside [0, %d)", t, T.pair_i, T.pair_j, N);
        } else if (T.kind != ADX_TERM_MACROSTATE) {
            return fail(ADX_EINVAL, "term %d: bad kind %d", t, T.kind);
        } else if (T.macrostate < 0 || T.macrostate >= d->n_macrostates) {
            return fail(ADX_EINVAL, "term %d names macrostate %d (have %d)", t, T.macrostate, d->n_macrostates);
        }
        if (T.condition != ADX_APO && T.condition != ADX_HOLO) return fail(ADX_EINVAL, "bad condition");
        c->terms.push_back(T);
    }
    if (d->fold_mode != ADX_FOLD_PF && d->fold_mode != ADX_FOLD_MFE) return fail(ADX_EINVAL, "bad fold_mode");
    pb.mode = d->fold_mode;
    c->thermo = d->thermostat;
    if (c->thermo.kind == ADX_THERMO_ANNEAL && c->thermo.cycle_len <= 0)
        return fail(ADX_EINVAL, "annealing cycle length must be positive");
    if (c->thermo.kind == ADX_THERMO_AUTO && c->thermo.period <= 0)
        return fail(ADX_EINVAL, "auto thermostat training period must be positive");
    if (c->thermo.kind < 0 || c->thermo.kind > 2) return fail(ADX_EINVAL, "bad thermostat kind");

    adx_status s = pb.init_device();
    if (s) return s;
    pb.Nraw = N;
    // motif
    if (d->aptamer_seq && d->aptamer_fold) {
        pb.motif.seq = d->aptamer_seq;
        for (auto &ch : pb.motif.seq) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
        pb.motif.fold = d->aptamer_fold;
        pb.motif.energy_kcal = d->aptamer_energy_kcal;
        pb.motif.mode = d->motif_mode;
        pb.motif.present = true;
        s = prepare_motif(*pb.P, pb.motif, pb.motif_eint, pb.motif_pt);
        if (s) return s;
    }
    // contexts (ScoreFunction::evaluate scoring.cc:123-132, map order)
    c->n_contexts = d->n_contexts;
    pb.n_ctx_eff = std::max(1, d->n_contexts);
    pb.n_terms = static_cast<int>(c->terms.size());
    pb.ctx_seq.clear();
    pb.ctx_off.clear();
    std::vector<int> ctxN;
    for (int k = 0; k < pb.n_ctx_eff; k++) {
        std::string b, a;
        if (d->n_contexts > 0) {
            b = d->contexts[k].before ? d->contexts[k].before : "";
            a = d->contexts[k].after ? d->contexts[k].after : "";
        }
        pb.ctx_off.push_back(static_cast<int>(pb.ctx_seq.size()));
        pb.ctx_off.push_back(static_cast<int>(b.size()));
        for (char ch : b) pb.ctx_seq.push_back(static_cast<uint8_t>(base_code(ch)));
        pb.ctx_off.push_back(static_cast<int>(pb.ctx_seq.size()));
        pb.ctx_off.push_back(static_cast<int>(a.size()));
        for (char ch : a) pb.ctx_seq.push_back(static_cast<uint8_t>(base_code(ch)));
        ctxN.push_back(static_cast<int>(b.size() + a.size()) + N);
    }
    if (pb.ctx_seq.empty()) pb.ctx_seq.push_back(0);
    pb.Nmax = *std::max_element(ctxN.begin(), ctxN.end());
    if (pb.Nmax > NMAX) return fail(ADX_EUNSUPPORTED, "folded length %d exceeds %d", pb.Nmax, NMAX);
    // variants: per context, (condition, macrostate | free); holo == apo without an aptamer
    std::map<std::tuple<int, int, int>, int> vindex;
    auto variant = [&](int ctx, int cond, int mac) -> int {
        if (!pb.motif.present) cond = ADX_APO;
        auto key = std::make_tuple(ctx, cond, mac);
        auto it = vindex.find(key);
        if (it != vindex.end()) return it->second;
        const int Nc = ctxN[ctx];
        std::string cst;
        if (mac >= 0) {
            const int lb = pb.ctx_off[4 * ctx + 1];
            cst = std::string(lb, '.') + c->macrostates[mac] + std::string(Nc - lb - N, '.');
        }
        std::vector<uint8_t> blob;
        adx_status st = build_constraint(cst, Nc, blob);
        if (st) return -1;
        DevVariant v{Nc, pb.ctx_off[4 * ctx + 1], d->n_contexts > 0 ? ctx : -1,
                     static_cast<int>(pb.cons.size()), cond == ADX_HOLO ? 1 : 0, 0};
        pb.cons.insert(pb.cons.end(), blob.begin(), blob.end());
        const int id = static_cast<int>(pb.variants.size());
        pb.variants.push_back(v);
        pb.vmac.push_back(mac);
        vindex[key] = id;
        return id;
    };
    variant(0, ADX_APO, -1);  // variant 0 = apo ensemble (calibration anchor)
    for (int k = 0; k < pb.n_ctx_eff; k++) {
        for (auto &T : c->terms) {
            const int vf = variant(k, T.condition, -1);
            if (T.kind == ADX_TERM_PAIR) {   // RnaFold::base_pair_prob of the unconstrained fold
                if (vf < 0) return ADX_ECONSTRAINT;
                int bv = -1;
                for (size_t b = 0; b < pb.bvars.size(); b++)
                    if (pb.bvars[b] == vf) bv = static_cast<int>(b);
                if (bv < 0) {
                    bv = static_cast<int>(pb.bvars.size());
                    pb.bvars.push_back(vf);
                }
                const int lb = pb.variants[vf].before_len;
                const int pidx = static_cast<int>(pb.pairs.size() / 3);
                pb.pairs.insert(pb.pairs.end(), {bv, T.pair_i + lb + 1, T.pair_j + lb + 1});
                DevTermMap m{vf, vf, T.favorable, T.weight};
                m.kind = 1;
                m.pidx = pidx;
                pb.tmap.push_back(m);
                continue;
            }
            const int vc = variant(k, T.condition, T.macrostate);
            if (vf < 0 || vc < 0) return ADX_ECONSTRAINT;
            pb.tmap.push_back(DevTermMap{vf, vc, T.favorable, T.weight});
        }
    }
    if (pb.tmap.empty()) pb.tmap.push_back(DevTermMap{0, 0, 1, 0.0});
    if (static_cast<int>(pb.variants.size()) > MAX_VARIANTS) return fail(ADX_EUNSUPPORTED, "too many fold variants");
    // moves: freely mutable positions and their closures
    for (int i = 0; i < N; i++) {
        bool free_ = std::isupper(static_cast<unsigned char>(c->templ[i])) != 0;
        for (auto &m : c->macrostates)
            if (m[i] == ')') free_ = false;
        if (free_) c->mut.push_back(i);
    }
    c->clo_off.push_back(0);
    for (int pos : c->mut) {
        std::vector<std::pair<int, int>> cl;
        const int rc = closure(c->templ, c->macrostates, pos, cl);
        c->clo_err.push_back(rc);
        if (rc == 0)
            for (auto &pp : cl) {
                c->clo_pos.push_back(pp.first);
                c->clo_par.push_back(static_cast<uint8_t>(pp.second));
            }
        c->clo_off.push_back(static_cast<int>(c->clo_pos.size()));
    }
    if (c->clo_pos.empty()) { c->clo_pos.push_back(0); c->clo_par.push_back(0); }
    s = pb.upload_all();
    if (s) return s;
    if (pb.mode == ADX_FOLD_PF) {   // the MFE tables carry no scale
        s = calibrate(pb, encode(c->templ));
        if (s) return s;
    }
    HIP_TRY(hipEventCreate(&c->ev0));
    HIP_TRY(hipEventCreate(&c->ev1));
    HIP_TRY(c->d_mut.upload(c->mut.data(), c->mut.size(), pb.stream));
    HIP_TRY(c->d_clo_off.upload(c->clo_off.data(), c->clo_off.size(), pb.stream));
    HIP_TRY(c->d_clo_pos.upload(c->clo_pos.data(), c->clo_pos.size(), pb.stream));
    HIP_TRY(c->d_clo_par.upload(c->clo_par.data(), c->clo_par.size(), pb.stream));
    HIP_TRY(c->d_clo_err.upload(c->clo_err.data(), c->clo_err.size(), pb.stream));
    HIP_TRY(hipStreamSynchronize(pb.stream));
    *out = c.release();
    return ADX_OK;
}

extern "C" void adx_ctx_destroy(adx_ctx *c) { delete c; }

extern "C" adx_status adx_ctx_info(const adx_ctx *c, adx_info *info) {
    if (!c || !info) return fail(ADX_EINVAL, "adx_ctx_info: null argument");
    info->length = c->pb.Nraw;
    info->n_variants = static_cast<int>(c->pb.variants.size());
    info->n_terms = c->pb.n_terms;
    info->n_mutable = static_cast<int>(c->mut.size());
    info->max_walkers = 1 << 24;
    info->scale_per_nt = c->pb.sigma();
    return ADX_OK;
}

extern "C" adx_status adx_variant_desc(const adx_ctx *c, int v, int *ctx, int *cond, int *mac) {
    if (!c || v < 0 || v >= static_cast<int>(c->pb.variants.size())) return fail(ADX_EINVAL, "bad variant");
    const DevVariant &V = c->pb.variants[v];
    if (ctx) *ctx = V.ctx;
    if (cond) *cond = V.motif ? ADX_HOLO : ADX_APO;
    if (mac) {
        *mac = -1;
        for (size_t t = 0; t < c->pb.tmap.size(); t++)
            if (c->pb.tmap[t].vcons == v && c->pb.n_terms > 0)
                *mac = c->terms[t % c->pb.n_terms].macrostate;
    }
    return ADX_OK;
}

static void mt_seed_host(uint32_t seed, uint32_t *mt) {
    mt[0] = seed;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    mt[624] = 624;
}

// Every walker's current configuration folded from scratch by the MC step's
// kernels (kernels.hip launch_rescore): fresh scores to prop_score, term
// values to dtv (device, optional), fresh tables adopted.
static adx_status rescore_walkers(adx_ctx *c, double *dtv) {
    Problem &pb = c->pb;
    const int W = c->W;
    adx_status s = pb.prepare(W);
    if (s) return s;
    StepArgs st{};
    st.cur_seq = c->cur_seq.p;
    st.prop_seq = c->prop_seq.p;
    st.prop_score = c->prop_score.p;
    st.changed = c->changed.p;
    st.Nraw = pb.Nraw;
    st.W = W;
    pb.state_on = true;
    const KArgs ka = pb.kargs();
    pb.state_on = false;
    HIP_TRY(launch_rescore(ka, st, dtv, pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_walkers_init(adx_ctx *c, int W, const char *seqs, const uint32_t *seeds) {
    if (!c || W <= 0 || !seeds) return fail(ADX_EINVAL, "adx_walkers_init: bad argument");
    Problem &pb = c->pb;
    const int N = pb.Nraw;
    if (c->mut.empty()) return fail(ADX_EMOVE, "no freely mutable positions (vector index out of range)");
    std::vector<uint8_t> codes(size_t(W) * N);
    for (int w = 0; w < W; w++)
        for (int k = 0; k < N; k++) {
            const char ch = seqs ? seqs[size_t(w) * N + k] : c->templ[k];
            codes[size_t(w) * N + k] = static_cast<uint8_t>(base_code(ch));
        }
    std::vector<uint32_t> mt(size_t(W) * MT_WORDS);
    for (int w = 0; w < W; w++) mt_seed_host(seeds[w], &mt[size_t(w) * MT_WORDS]);
    c->W = W;
    c->step = 0;
    HIP_TRY(c->cur_seq.upload(codes.data(), codes.size(), pb.stream));
    HIP_TRY(c->mtA.upload(mt.data(), mt.size(), pb.stream));
    HIP_TRY(c->mtC.upload(mt.data(), mt.size(), pb.stream));
    HIP_TRY(c->cur_score.alloc(W));
    HIP_TRY(c->last_diff.alloc(W));
    HIP_TRY(c->auto_T.alloc(W));
    HIP_TRY(c->counters.alloc(size_t(W) * 4));
    HIP_TRY(c->ntrain.alloc(W));
    HIP_TRY(c->err.alloc(W));
    HIP_TRY(c->prop_seq.alloc(size_t(W) * N));
    HIP_TRY(c->prop_score.alloc(W));
    HIP_TRY(c->temp.alloc(W));
    HIP_TRY(c->u.alloc(W));
    HIP_TRY(c->changed.alloc(W));
    HIP_TRY(c->pick.alloc(W));
    HIP_TRY(c->bcode.alloc(W));
    const int period = std::max(1, c->thermo.period);
    HIP_TRY(c->train.alloc(c->thermo.kind == ADX_THERMO_AUTO ? size_t(W) * period : 1));
    HIP_TRY(hipMemsetAsync(c->last_diff.p, 0, sizeof(double) * W, pb.stream));
    HIP_TRY(hipMemsetAsync(c->counters.p, 0, sizeof(int64_t) * W * 4, pb.stream));
    HIP_TRY(hipMemsetAsync(c->ntrain.p, 0, sizeof(int) * W, pb.stream));
    HIP_TRY(hipMemsetAsync(c->err.p, 0, sizeof(int) * W, pb.stream));
    std::vector<double> t0(W, c->thermo.t_init);
    HIP_TRY(hipMemcpyAsync(c->auto_T.p, t0.data(), sizeof(double) * W, hipMemcpyHostToDevice, pb.stream));
    // initial score (sampling.cc:40) with the MC step's own kernels; it also
    // stores the walkers' first tables
    adx_status s = pb.alloc_state(W);
    if (s) return s;
    s = rescore_walkers(c, nullptr);
    if (s) return s;
    HIP_TRY(hipMemcpyAsync(c->cur_score.p, c->prop_score.p, sizeof(double) * W, hipMemcpyDeviceToDevice, pb.stream));
    HIP_TRY(hipStreamSynchronize(pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_walkers_rescore(adx_ctx *c, double *scores, double *term_values) {
    if (!c || !scores) return fail(ADX_EINVAL, "adx_walkers_rescore: null argument");
    if (c->W <= 0) return fail(ADX_ESTATE, "adx_walkers_rescore before adx_walkers_init");
    Problem &pb = c->pb;
    const int W = c->W, ntt = pb.n_terms * pb.n_ctx_eff;
    DevBuf<double> dtv;
    if (term_values && ntt > 0) HIP_TRY(dtv.alloc(size_t(W) * ntt));
    adx_status s = rescore_walkers(c, dtv.p);
    if (s) return s;
    HIP_TRY(hipMemcpyAsync(scores, c->prop_score.p, sizeof(double) * W, hipMemcpyDeviceToHost, pb.stream));
    if (dtv.p)
        HIP_TRY(hipMemcpyAsync(term_values, dtv.p, sizeof(double) * W * ntt, hipMemcpyDeviceToHost, pb.stream));
    HIP_TRY(hipStreamSynchronize(pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_run_steps(adx_ctx *c, int steps, adx_trace *trace) {
    if (!c) return fail(ADX_EINVAL, "adx_run_steps: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "adx_run_steps before adx_walkers_init");
    if (steps <= 0) return ADX_OK;
    Problem &pb = c->pb;
    StepArgs st{};
    st.cur_seq = c->cur_seq.p;
    st.cur_score = c->cur_score.p;
    st.mtA = c->mtA.p;
    st.mtC = c->mtC.p;
    st.counters = c->counters.p;
    st.last_diff = c->last_diff.p;
    st.auto_T = c->auto_T.p;
    st.train = c->train.p;
    st.ntrain = c->ntrain.p;
    st.err = c->err.p;
    st.prop_seq = c->prop_seq.p;
    st.prop_score = c->prop_score.p;
    st.changed = c->changed.p;
    st.chg = c->pb.dChg.p;
    st.pick = c->pick.p;
    st.bcode = c->bcode.p;
    st.temp = c->temp.p;
    st.u = c->u.p;
    st.Nraw = pb.Nraw;
    st.mut = c->d_mut.p;
    st.clo_off = c->d_clo_off.p;
    st.clo_pos = c->d_clo_pos.p;
    st.clo_par = c->d_clo_par.p;
    st.clo_err = c->d_clo_err.p;
    st.M = static_cast<int>(c->mut.size());
    st.thermo_kind = c->thermo.kind;
    st.t_fixed = c->thermo.t_fixed;
    st.t_hi = c->thermo.t_hi;
    st.t_lo = c->thermo.t_lo;
    st.cycle_len = std::max(1, c->thermo.cycle_len);
    st.ln_target_rate = std::log(c->thermo.target_rate);
    st.period = std::max(1, c->thermo.period);
    st.step0 = c->step;
    st.nsteps = steps;
    st.W = c->W;
    const int W = c->W;
    const int ntt = pb.n_terms * pb.n_ctx_eff;
    DevBuf<int32_t> tpos, tout;
    DevBuf<int8_t> tbase;
    DevBuf<double> ttemp, tprop, tcur, tu, tterms;
    const size_t R = size_t(steps) * W;
    if (trace) {
        HIP_TRY(tpos.alloc(R));
        HIP_TRY(tout.alloc(R));
        HIP_TRY(tbase.alloc(R));
        HIP_TRY(ttemp.alloc(R));
        HIP_TRY(tprop.alloc(R));
        HIP_TRY(tcur.alloc(R));
        HIP_TRY(tu.alloc(R));
        HIP_TRY(tterms.alloc(R * std::max(1, ntt)));
        st.tr_pos = tpos.p;
        st.tr_outcome = tout.p;
        st.tr_base = tbase.p;
        st.tr_temp = ttemp.p;
        st.tr_prop = tprop.p;
        st.tr_cur = tcur.p;
        st.tr_u = tu.p;
        st.tr_terms = ntt > 0 ? tterms.p : nullptr;
    }
    // events around every score window (the dominant kernels) for its average duration
    std::vector<hipEvent_t> evs(4 * size_t(steps));
    for (auto &e : evs) HIP_TRY(hipEventCreate(&e));
    struct EvFree {
        std::vector<hipEvent_t> &v;
        ~EvFree() { for (auto e : v) (void)hipEventDestroy(e); }
    } evfree{evs};
    HIP_TRY(hipEventRecord(c->ev0, pb.stream));
    pb.state_on = true;   // incremental folds against the walkers' stored tables
    const KArgs ka_steps = pb.kargs();
    pb.state_on = false;
    c->inside_kernel = inside_kernel_name(ka_steps);
    c->outside_kernel = outside_kernel_name(ka_steps);
    HIP_TRY(launch_steps(ka_steps, pb.qbm, st, pb.stream, evs.data()));
    HIP_TRY(hipEventRecord(c->ev1, pb.stream));
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->last_ms = ms;
    double sk = 0.0, si = 0.0, so = 0.0;
    for (int k = 0; k < steps; k++) {
        float e = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&e, evs[4 * k], evs[4 * k + 3]));
        HIP_TRY(hipEventElapsedTime(&b, evs[4 * k + 1], evs[4 * k + 2]));
        sk += e;
        si += e - b;   // the window minus its outside pass (kernels.hip launch_steps)
        so += b;
    }
    c->score_ms_total = sk;
    c->inside_ms_total = si;
    c->outside_ms_total = so;
    c->score_launches = steps;
    c->step += steps;
    std::vector<int> errs(W);
    HIP_TRY(hipMemcpy(errs.data(), c->err.p, sizeof(int) * W, hipMemcpyDeviceToHost));
    if (trace) {
        std::vector<int8_t> b(R);
        if (trace->position) HIP_TRY(hipMemcpy(trace->position, tpos.p, R * 4, hipMemcpyDeviceToHost));
        if (trace->outcome) HIP_TRY(hipMemcpy(trace->outcome, tout.p, R * 4, hipMemcpyDeviceToHost));
        if (trace->base) {
            HIP_TRY(hipMemcpy(b.data(), tbase.p, R, hipMemcpyDeviceToHost));
            for (size_t k = 0; k < R; k++) trace->base[k] = b[k] >= 1 && b[k] <= 4 ? "ACGU"[b[k] - 1] : 'N';
        }
        if (trace->temperature) HIP_TRY(hipMemcpy(trace->temperature, ttemp.p, R * 8, hipMemcpyDeviceToHost));
        if (trace->proposed_score) HIP_TRY(hipMemcpy(trace->proposed_score, tprop.p, R * 8, hipMemcpyDeviceToHost));
        if (trace->current_score) HIP_TRY(hipMemcpy(trace->current_score, tcur.p, R * 8, hipMemcpyDeviceToHost));
        if (trace->random_threshold) HIP_TRY(hipMemcpy(trace->random_threshold, tu.p, R * 8, hipMemcpyDeviceToHost));
        if (trace->term_values && ntt > 0)
            HIP_TRY(hipMemcpy(trace->term_values, tterms.p, R * ntt * 8, hipMemcpyDeviceToHost));
    }
    for (int w = 0; w < W; w++)
        if (errs[w]) return fail(ADX_EMOVE, "walker %d: %s", w, move_error_text(errs[w]));
    return ADX_OK;
}

extern "C" adx_status adx_last_kernel_ms(const adx_ctx *c, double *ms) {
    if (!c || !ms) return fail(ADX_EINVAL, "adx_last_kernel_ms: null argument");
    *ms = c->last_ms;
    return ADX_OK;
}

extern "C" adx_status adx_last_score_kernel_ms(const adx_ctx *c, double *avg_ms, int *launches) {
    if (!c || !avg_ms) return fail(ADX_EINVAL, "adx_last_score_kernel_ms: null argument");
    *avg_ms = c->score_launches ? c->score_ms_total / c->score_launches : 0.0;
    if (launches) *launches = c->score_launches;
    return ADX_OK;
}

extern "C" adx_status adx_last_kernel_split_ms(const adx_ctx *c, double *inside_ms, double *outside_ms) {
    if (!c || !inside_ms || !outside_ms) return fail(ADX_EINVAL, "adx_last_kernel_split_ms: null argument");
    const int n = c->score_launches;
    *inside_ms = n ? c->inside_ms_total / n : 0.0;
    *outside_ms = n ? c->outside_ms_total / n : 0.0;
    return ADX_OK;
}

extern "C" adx_status adx_last_kernel_names(const adx_ctx *c, char *inside, int inside_len, char *outside,
                                            int outside_len) {
    if (!c || !inside || !outside || inside_len <= 0 || outside_len <= 0)
        return fail(ADX_EINVAL, "adx_last_kernel_names: bad argument");
    std::snprintf(inside, size_t(inside_len), "%s", c->inside_kernel.c_str());
    std::snprintf(outside, size_t(outside_len), "%s", c->outside_kernel.c_str());
    return ADX_OK;
}

extern "C" adx_status adx_walkers_download(adx_ctx *c, char *seqs, double *scores, int64_t *counters) {
    if (!c) return fail(ADX_EINVAL, "adx_walkers_download: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "no walkers");
    const int W = c->W, N = c->pb.Nraw;
    HIP_TRY(hipStreamSynchronize(c->pb.stream));
    if (seqs) {
        std::vector<uint8_t> codes(size_t(W) * N);
        HIP_TRY(hipMemcpy(codes.data(), c->cur_seq.p, codes.size(), hipMemcpyDeviceToHost));
        for (int w = 0; w < W; w++)
            for (int k = 0; k < N; k++) {
                const uint8_t b = codes[size_t(w) * N + k];
                char ch = b >= 1 && b <= 4 ? "ACGU"[b - 1] : 'N';
                if (std::islower(static_cast<unsigned char>(c->templ[k])))
                    ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
                seqs[size_t(w) * N + k] = ch;
            }
    }
    if (scores) HIP_TRY(hipMemcpy(scores, c->cur_score.p, sizeof(double) * W, hipMemcpyDeviceToHost));
    if (counters) HIP_TRY(hipMemcpy(counters, c->counters.p, sizeof(int64_t) * W * 4, hipMemcpyDeviceToHost));
    return ADX_OK;
}

extern "C" adx_status adx_walkers_export(adx_ctx *c, void *dev_seqs, void *dev_scores) {
    if (!c) return fail(ADX_EINVAL, "adx_walkers_export: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "no walkers");
    const size_t W = size_t(c->W), N = size_t(c->pb.Nraw);
    if (dev_seqs) HIP_TRY(hipMemcpyAsync(dev_seqs, c->cur_seq.p, W * N, hipMemcpyDeviceToDevice, c->pb.stream));
    if (dev_scores)
        HIP_TRY(hipMemcpyAsync(dev_scores, c->cur_score.p, W * sizeof(double), hipMemcpyDeviceToDevice, c->pb.stream));
    HIP_TRY(hipStreamSynchronize(c->pb.stream));
    return ADX_OK;
}

// `a` waits (on the device) for the work queued on `b` so far
static hipError_t stream_after(hipStream_t a, hipStream_t b) {
    hipEvent_t ev;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ev, b);
    if (e == hipSuccess) e = hipStreamWaitEvent(a, ev, 0);
    (void)hipEventDestroy(ev);
    return e;
}

extern "C" adx_status adx_walkers_export_on(adx_ctx *c, void *dev_seqs, void *dev_scores, void *stream) {
    if (!c) return fail(ADX_EINVAL, "adx_walkers_export_on: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "no walkers");
    const size_t W = size_t(c->W), N = size_t(c->pb.Nraw);
    const hipStream_t other = hipStream_t(stream);   // NULL: the null stream, a valid handle
    // the caller's earlier reads of the buffers finish before the copies overwrite them
    HIP_TRY(stream_after(c->pb.stream, other));
    if (dev_seqs) HIP_TRY(hipMemcpyAsync(dev_seqs, c->cur_seq.p, W * N, hipMemcpyDeviceToDevice, c->pb.stream));
    if (dev_scores)
        HIP_TRY(hipMemcpyAsync(dev_scores, c->cur_score.p, W * sizeof(double), hipMemcpyDeviceToDevice, c->pb.stream));
    // and the caller's later work on `stream` sees them
    HIP_TRY(stream_after(other, c->pb.stream));
    return ADX_OK;
}

// The copies and resets of an import, queued on the engine stream (both import
// entry points: they differ only in how they order against the caller)
static hipError_t import_queue(adx_ctx *c, const void *dev_seqs, const void *dev_scores) {
    const size_t W = size_t(c->W), N = size_t(c->pb.Nraw);
    hipError_t e = hipSuccess;
    if (dev_seqs) e = hipMemcpyAsync(c->cur_seq.p, dev_seqs, W * N, hipMemcpyDeviceToDevice, c->pb.stream);
    if (e == hipSuccess && dev_scores)
        e = hipMemcpyAsync(c->cur_score.p, dev_scores, W * sizeof(double), hipMemcpyDeviceToDevice, c->pb.stream);
    if (e == hipSuccess && dev_seqs && c->pb.dValid.p)   // new configurations: their next fold starts from scratch
        e = hipMemsetAsync(c->pb.dValid.p, 0, W, c->pb.stream);
    return e;
}

extern "C" adx_status adx_walkers_import_after(adx_ctx *c, const void *dev_seqs, const void *dev_scores,
                                               void *producer_stream) {
    if (!c) return fail(ADX_EINVAL, "adx_walkers_import_after: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "no walkers");
    // NULL is the null stream (torch's default stream), not "no producer": the
    // engine stream is non-blocking and would not otherwise wait for it
    const hipStream_t other = hipStream_t(producer_stream);
    HIP_TRY(stream_after(c->pb.stream, other));
    HIP_TRY(import_queue(c, dev_seqs, dev_scores));
    // the producer's later writes to the buffers wait for the copies
    HIP_TRY(stream_after(other, c->pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_walkers_import(adx_ctx *c, const void *dev_seqs, const void *dev_scores) {
    if (!c) return fail(ADX_EINVAL, "adx_walkers_import: null context");
    if (c->W <= 0) return fail(ADX_ESTATE, "no walkers");
    HIP_TRY(import_queue(c, dev_seqs, dev_scores));
    HIP_TRY(hipStreamSynchronize(c->pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_set_temperature(adx_ctx *c, double t) {
    if (!c) return fail(ADX_EINVAL, "adx_set_temperature: null context");
    if (c->thermo.kind != ADX_THERMO_FIXED) return fail(ADX_EINVAL, "adx_set_temperature: not a fixed thermostat");
    c->thermo.t_fixed = t;
    return ADX_OK;
}

extern "C" adx_status adx_bppm_batch(adx_ctx *c, int W, const char *seqs, int condition, int context,
                                      double *probs) {
    if (!c || W <= 0 || !seqs || !probs) return fail(ADX_EINVAL, "adx_bppm_batch: bad argument");
    Problem &pb = c->pb;
    if (pb.mode != ADX_FOLD_PF) return fail(ADX_EUNSUPPORTED, "adx_bppm_batch: partition-function contexts only");
    const int want_ctx = c->n_contexts > 0 ? context : -1;
    int v = -1;
    for (size_t k = 0; k < pb.variants.size(); k++)
        if (pb.variants[k].ctx == want_ctx && pb.vmac[k] == -1 && pb.variants[k].motif == (condition == ADX_HOLO ? 1 : 0))
            v = static_cast<int>(k);
    if (v < 0) return fail(ADX_EINVAL, "adx_bppm_batch: the objective has no (context %d, condition %d) fold", context, condition);
    const int N = pb.Nraw, L = pb.variants[v].N;
    std::vector<uint8_t> codes(size_t(W) * N);
    for (size_t k = 0; k < codes.size(); k++) codes[k] = static_cast<uint8_t>(base_code(seqs[k]));
    DevBuf<uint8_t> dseq;
    DevBuf<int> dbv;
    DevBuf<double> dfull;
    HIP_TRY(dseq.upload(codes.data(), codes.size(), pb.stream));
    HIP_TRY(dbv.upload(&v, 1, pb.stream));
    KArgs ka = pb.kargs();
    ka.bvars = dbv.p;
    ka.n_bvars = 1;
    ka.bvar_slot = nullptr;   // no stored tables are reused here
    ka.n_pairs = 0;
    ka.pairs = nullptr;
    ka.pair_p = nullptr;
    if (bppm_lds_bytes(ka, nullptr) == 0)
        return fail(ADX_EUNSUPPORTED, "base-pair probabilities of length %d do not fit one CU's LDS yet", pb.Nmax);
    DevBuf<char> dscr;
    const size_t scr = bppm_scratch_bytes(ka, W);
    if (scr) HIP_TRY(dscr.alloc(scr));
    ka.bppm_scratch = dscr.p;
    HIP_TRY(dfull.alloc(size_t(W) * L * L));
    HIP_TRY(hipMemsetAsync(dfull.p, 0, sizeof(double) * W * L * L, pb.stream));
    HIP_TRY(launch_bppm(ka, dseq.p, W, nullptr, dfull.p, L, nullptr, ka.bppm_scratch, pb.stream));
    HIP_TRY(hipMemcpyAsync(probs, dfull.p, sizeof(double) * W * L * L, hipMemcpyDeviceToHost, pb.stream));
    HIP_TRY(hipStreamSynchronize(pb.stream));
    return ADX_OK;
}

extern "C" adx_status adx_score_batch(adx_ctx *c, int W, const char *seqs, double *scores,
                                      double *term_values, float *dG) {
    if (!c || W <= 0 || !seqs || !scores) return fail(ADX_EINVAL, "adx_score_batch: bad argument");
    Problem &pb = c->pb;
    const int N = pb.Nraw;
    std::vector<uint8_t> codes(size_t(W) * N);
    for (size_t k = 0; k < codes.size(); k++) codes[k] = static_cast<uint8_t>(base_code(seqs[k]));
    const int V = static_cast<int>(pb.variants.size());
    const int ntt = pb.n_terms * pb.n_ctx_eff;
    DevBuf<uint8_t> dseq;
    DevBuf<double> dsc, dterms;
    DevBuf<float> ddg;
    HIP_TRY(dseq.upload(codes.data(), codes.size(), pb.stream));
    HIP_TRY(dsc.alloc(W));
    HIP_TRY(dterms.alloc(size_t(W) * std::max(1, ntt)));
    HIP_TRY(ddg.alloc(size_t(W) * V));
    HIP_TRY(hipEventRecord(c->ev0, pb.stream));
    adx_status s = pb.score(dseq.p, W, dsc.p, ntt > 0 ? dterms.p : nullptr, ddg.p);
    if (s) return s;
    HIP_TRY(hipEventRecord(c->ev1, pb.stream));
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->last_ms = ms;
    HIP_TRY(hipMemcpy(scores, dsc.p, sizeof(double) * W, hipMemcpyDeviceToHost));
    if (term_values && ntt > 0)
        HIP_TRY(hipMemcpy(term_values, dterms.p, sizeof(double) * W * ntt, hipMemcpyDeviceToHost));
    if (dG) HIP_TRY(hipMemcpy(dG, ddg.p, sizeof(float) * W * V, hipMemcpyDeviceToHost));
    return ADX_OK;
}
