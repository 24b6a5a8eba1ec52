/* CPU restatement of the ViennaRNA-2.x energy model + McCaskill partition
 * function as driven by addapt (TEST INFRASTRUCTURE ONLY).
 *
 * Call sites restated: ViennaRnaFold::macrostate_prob / make_fold_compound
 * (/root/reference/src/scoring.cc:53-103) and base_pair_prob (:37-51).
 * ViennaRNA itself (the third-party dependency holding the arithmetic, version
 * unpinned by /root/reference/configure.ac:27-30, API era 2.2.x) is not
 * vendored; the recursions below restate its published default model:
 *   E_Hairpin / E_IntLoop / E_ExtLoop / E_MLstem, dangles = 2, TURN = 3,
 *   MAXLOOP = 30, special hairpins, pf over qb/qm/qm1/q with hard
 *   constraints from dot-bracket strings (DB_DEFAULT | ENFORCE_BP).
 * Everything here is plain double precision with no pf_scale, so it checks
 * the GPU path's scaled FP32 arithmetic independently. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "adx_oracle.h"

#define IDX(i, j) ((size_t)(i) * (size_t)(N + 2) + (size_t)(j))

static const int PAIR[5][5] = {
    /*      N  A  C  G  U */
    /* N */ {0, 0, 0, 0, 0},
    /* A */ {0, 0, 0, 0, 5},
    /* C */ {0, 0, 0, 1, 0},
    /* G */ {0, 0, 2, 0, 3},
    /* U */ {0, 6, 0, 4, 0}};
static const int RTYPE[8] = {0, 2, 1, 4, 3, 6, 5, 7};

static int enc_base(char c) {
    switch (c) {
    case 'A': case 'a': return 1;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 3;
    case 'U': case 'u': case 'T': case 't': return 4;
    default: return 0;
    }
}

static double boltz(double e_dcal) { return exp(-e_dcal * 10.0 / orc_kT_cal()); }

/* ---------------------------------------------------------------- energies */
static double E_hairpin(const orc_params *P, int i, int j, const int *S, const char *useq) {
    int u = j - i - 1;
    int type = PAIR[S[i]][S[j]];
    double e = (u <= 30) ? P->hairpin[u] : P->hairpin[30] + P->lxc * log(u / 30.0);
    if (u < 3) return e;
    if (u == 4) {
        for (int k = 0; k < P->ntetra; k++)
            if (strncmp(useq + i, P->tetra[k], 6) == 0) return P->tetraE[k];
    } else if (u == 6) {
        for (int k = 0; k < P->nhexa; k++)
            if (strncmp(useq + i, P->hexa[k], 8) == 0) return P->hexaE[k];
    } else if (u == 3) {
        for (int k = 0; k < P->ntri; k++)
            if (strncmp(useq + i, P->tri[k], 5) == 0) return P->triE[k];
        return e + (type > 2 ? P->TermAU : 0);
    }
    return e + P->mmH[type][S[i + 1]][S[j - 1]];
}

/* E_IntLoop(n1, n2, type, type_2, si1, sj1, sp1, sq1): type_2 = type of the
 * reversed inner pair (q,p). */
static double E_int(const orc_params *P, int n1, int n2, int type, int type_2, int si1, int sj1,
                    int sp1, int sq1) {
    int nl = n1 > n2 ? n1 : n2, ns = n1 > n2 ? n2 : n1;
    double e;
    if (nl == 0) return P->stack[type][type_2];
    if (ns == 0) {
        e = (nl <= ORC_MAXLOOP) ? P->bulge[nl] : P->bulge[30] + P->lxc * log(nl / 30.0);
        if (nl == 1) e += P->stack[type][type_2];
        else {
            if (type > 2) e += P->TermAU;
            if (type_2 > 2) e += P->TermAU;
        }
        return e;
    }
    if (ns == 1) {
        if (nl == 1) return P->int11[type][type_2][si1][sj1];
        if (nl == 2) {
            if (n1 == 1) return P->int21[type][type_2][si1][sq1][sj1];
            return P->int21[type_2][type][sq1][si1][sp1];
        }
        e = (nl + 1 <= ORC_MAXLOOP) ? P->interior[nl + 1]
                                    : P->interior[30] + P->lxc * log((nl + 1) / 30.0);
        int nin = (nl - ns) * P->ninio;
        e += (nin < P->maxninio) ? nin : P->maxninio;
        e += P->mm1nI[type][si1][sj1] + P->mm1nI[type_2][sq1][sp1];
        return e;
    }
    if (ns == 2) {
        if (nl == 2) return P->int22[type][type_2][si1][sp1][sq1][sj1];
        if (nl == 3) {
            e = P->interior[5] + P->ninio;
            e += P->mm23I[type][si1][sj1] + P->mm23I[type_2][sq1][sp1];
            return e;
        }
    }
    int u = nl + ns;
    e = (u <= ORC_MAXLOOP) ? P->interior[u] : P->interior[30] + P->lxc * log(u / 30.0);
    int nin = (nl - ns) * P->ninio;
    e += (nin < P->maxninio) ? nin : P->maxninio;
    e += P->mmI[type][si1][sj1] + P->mmI[type_2][sq1][sp1];
    return e;
}

static int E_ext_stem(const orc_params *P, int type, int n5d, int n3d) {
    int e = 0;
    if (n5d >= 0 && n3d >= 0) e += P->mmExt[type][n5d][n3d];
    else if (n5d >= 0) e += P->d5[type][n5d];
    else if (n3d >= 0) e += P->d3[type][n3d];
    if (type > 2) e += P->TermAU;
    return e;
}

static int E_ml_stem(const orc_params *P, int type, int n5d, int n3d) {
    int e = 0;
    if (n5d >= 0 && n3d >= 0) e += P->mmM[type][n5d][n3d];
    else if (n5d >= 0) e += P->d5[type][n5d];
    else if (n3d >= 0) e += P->d3[type][n3d];
    if (type > 2) e += P->TermAU;
    return e + P->MLintern;
}

/* ----------------------------------------------------------- constraints */
typedef struct {
    int N;
    unsigned char *allowed; /* (N+2)^2, sequence-independent part */
    int *up;                /* consecutive unpaired-allowed run from i */
    int ok;
} hc_t;

/* Dot-bracket hard constraint, DB_DEFAULT | ENFORCE_BP (scoring.cc:61-62):
 * '.' free, 'x' unpaired, '|' paired, '<' paired upstream (j < i),
 * '>' paired downstream (j > i), '()' enforced pair; crossing pairs of an
 * enforced pair are forbidden.  Unknown characters are treated as '.'. */
static hc_t build_hc(int N, const char *cst) {
    hc_t h;
    h.N = N;
    h.ok = 1;
    h.allowed = (unsigned char *)calloc((size_t)(N + 2) * (N + 2), 1);
    h.up = (int *)calloc(N + 3, sizeof(int));
    int *partner = (int *)malloc(sizeof(int) * (N + 2));
    int *enc = (int *)malloc(sizeof(int) * (N + 2));
    int *unp = (int *)malloc(sizeof(int) * (N + 2));
    int *stk = (int *)malloc(sizeof(int) * (N + 2));
    for (int i = 0; i <= N + 1; i++) { partner[i] = -1; enc[i] = 0; unp[i] = 1; }
    int sp = 0;
    for (int i = 1; i <= N; i++) {
        char c = cst ? cst[i - 1] : '.';
        enc[i] = sp ? stk[sp - 1] : 0;
        if (c == '(') { stk[sp++] = i; }
        else if (c == ')') {
            if (!sp) { h.ok = 0; break; }
            int a = stk[--sp];
            partner[a] = i;
            partner[i] = a;
            enc[i] = sp ? stk[sp - 1] : 0;
        }
    }
    if (sp) h.ok = 0;
    for (int i = 1; i <= N; i++) {
        char c = cst ? cst[i - 1] : '.';
        if (c == '|' || c == '<' || c == '>' || partner[i] >= 0) unp[i] = 0;
    }
    for (int i = 1; i <= N; i++) {
        char ci = cst ? cst[i - 1] : '.';
        for (int j = i + ORC_TURN + 1; j <= N; j++) {
            char cj = cst ? cst[j - 1] : '.';
            int a = 1;
            if (ci == 'x' || cj == 'x') a = 0;
            if (ci == '<' || cj == '>') a = 0;
            if (partner[i] >= 0 && partner[i] != j) a = 0;
            if (partner[j] >= 0 && partner[j] != i) a = 0;
            if (a && partner[i] < 0 && partner[j] < 0 && enc[i] != enc[j]) a = 0;
            h.allowed[IDX(i, j)] = (unsigned char)a;
        }
    }
    h.up[N + 1] = 0;
    for (int i = N; i >= 1; i--) h.up[i] = unp[i] ? h.up[i + 1] + 1 : 0;
    free(partner); free(enc); free(unp); free(stk);
    return h;
}

static void free_hc(hc_t *h) { free(h->allowed); free(h->up); }

/* ------------------------------------------------------------- the model */
typedef struct {
    const orc_params *P;
    int N;
    int *S;     /* 0..N+1, S[0] = S[N], S[N+1] = S[1] (ViennaRNA S1 wrap) */
    char *useq; /* 1-based upper-case copy, useq[0] = ' ' */
    hc_t hc;
    /* motif */
    int mL;
    int *mpt;   /* motif pair table (0-based, -1 unpaired) */
    const char *mseq;
    double m_extra; /* Boltzmann extra weight for a formed motif (unscaled) */
    double m_Eint;
    double m_beff;  /* PF bonus applied to the formed motif (kcal; mode REPLACE: minus Eint) */
    int m_mfe_dcal; /* motif structure energy incl. bonus for the MFE, lround(100*(Eint+beff)) */
} model_t;

static int can_pair(const model_t *m, int i, int j) {
    if (j - i < ORC_TURN + 1) return 0;
    int t = PAIR[m->S[i]][m->S[j]];
    return t && m->hc.allowed[(size_t)i * (size_t)(m->N + 2) + (size_t)j];
}

static void model_free(model_t *m) {
    free(m->S);
    free(m->useq);
    free(m->mpt);
    free_hc(&m->hc);
}

double orc_eval_structure(const orc_params *P, const char *seq, const char *structure);

static int model_init(model_t *m, const orc_params *P, const char *seq, const char *cst,
                      const orc_motif *motif) {
    memset(m, 0, sizeof *m);
    int N = (int)strlen(seq);
    m->P = P;
    m->N = N;
    m->S = (int *)malloc(sizeof(int) * (N + 2));
    m->useq = (char *)malloc(N + 2);
    m->useq[0] = ' ';
    for (int i = 1; i <= N; i++) {
        m->S[i] = enc_base(seq[i - 1]);
        char c = seq[i - 1];
        if (c >= 'a' && c <= 'z') c = (char)(c - 32);
        if (c == 'T') c = 'U';
        m->useq[i] = c;
    }
    m->useq[N + 1] = 0;
    m->S[0] = N ? m->S[N] : 0;
    m->S[N + 1] = N ? m->S[1] : 0;
    m->hc = build_hc(N, cst);
    if (!m->hc.ok) return 0;
    m->mL = 0;
    if (motif && motif->seq && motif->fold) {
        int L = (int)strlen(motif->seq);
        m->mL = L;
        m->mseq = motif->seq;
        m->mpt = (int *)malloc(sizeof(int) * L);
        int *stk = (int *)malloc(sizeof(int) * L), sp = 0;
        for (int k = 0; k < L; k++) m->mpt[k] = -1;
        for (int k = 0; k < L; k++) {
            if (motif->fold[k] == '(') stk[sp++] = k;
            else if (motif->fold[k] == ')' && sp) {
                int a = stk[--sp];
                m->mpt[a] = k;
                m->mpt[k] = a;
            }
        }
        free(stk);
        double eint = orc_eval_structure(P, motif->seq, motif->fold); /* kcal */
        m->m_Eint = eint;
        /* mode 0 (AUTO, the default): ADD for partition functions (bonus + the
         * motif's own loops: the ensemble annotations, test_scoring.cc:54-55),
         * REPLACE for the MFE (motif energy := bonus: the printed holo MFE
         * -9.22, test_scoring.cc:152-154); mode 1 (ADD) and mode 2 (REPLACE)
         * apply one reading to both fold modes */
        double beff = motif->mode == 2 ? motif->energy_kcal - eint : motif->energy_kcal;
        double beff_mfe = motif->mode == 1 ? motif->energy_kcal : motif->energy_kcal - eint;
        m->m_extra = boltz(eint * 100.0) * (boltz(beff * 100.0) - 1.0);
        m->m_beff = beff;
        m->m_mfe_dcal = (int)lround(100.0 * (eint + beff_mfe));
    }
    return 1;
}

/* Is the motif formed-able with its outer pair at (i, i+L-1)? */
static int motif_at(const model_t *m, int i, int j) {
    if (!m->mL || j - i + 1 != m->mL) return 0;
    for (int k = 0; k < m->mL; k++) {
        char c = m->mseq[k];
        if (c >= 'a' && c <= 'z') c = (char)(c - 32);
        if (m->useq[i + k] != c) return 0;
    }
    if (m->mpt[0] != m->mL - 1) return 0;
    const int N = m->N;
    for (int k = 0; k < m->mL; k++) {
        int pk = m->mpt[k];
        if (pk < 0) {
            if (m->hc.up[i + k] < 1) return 0;
        } else if (pk > k) {
            int a = i + k, b = i + pk;
            if (!PAIR[m->S[a]][m->S[b]] || !m->hc.allowed[IDX(a, b)]) return 0;
        }
    }
    return 1;
}

/* ------------------------------------------------------- inside (pf) */
typedef struct {
    double *qb, *qm, *qm1, *q5;
    double *stemM;  /* ML stem Boltzmann factor per (i,j) */
} pf_tables;

static double pf_inside(const model_t *m, pf_tables *T, int64_t *nint, int64_t *nml) {
    const orc_params *P = m->P;
    const int N = m->N;
    const int *S = m->S;
    const int *up = m->hc.up;
    size_t sz = (size_t)(N + 2) * (N + 2);
    T->qb = (double *)calloc(sz, sizeof(double));
    T->qm = (double *)calloc(sz, sizeof(double));
    T->qm1 = (double *)calloc(sz, sizeof(double));
    T->stemM = (double *)calloc(sz, sizeof(double));
    T->q5 = (double *)calloc(N + 2, sizeof(double));
    double *qb = T->qb, *qm = T->qm, *qm1 = T->qm1;
    double eMLbase = boltz(P->MLbase);
    int64_t ci = 0, cm = 0;
    for (int d = ORC_TURN + 1; d <= N - 1; d++) {
        for (int i = 1; i + d <= N; i++) {
            int j = i + d;
            double qbt = 0.0;
            if (can_pair(m, i, j)) {
                int type = PAIR[S[i]][S[j]];
                int u = j - i - 1;
                if (up[i + 1] >= u) qbt += boltz(E_hairpin(P, i, j, S, m->useq));
                for (int p = i + 1; p <= i + ORC_MAXLOOP + 1 && p < j - ORC_TURN - 1; p++) {
                    int n1 = p - i - 1;
                    if (n1 > 0 && up[i + 1] < n1) break;
                    int minq = j - 1 - (ORC_MAXLOOP - n1);
                    if (minq < p + ORC_TURN + 1) minq = p + ORC_TURN + 1;
                    for (int q = j - 1; q >= minq; q--) {
                        int n2 = j - q - 1;
                        if (n2 > 0 && up[q + 1] < n2) break;
                        if (!can_pair(m, p, q)) continue;
                        int type2 = PAIR[S[q]][S[p]];
                        ci++;
                        qbt += qb[IDX(p, q)] *
                               boltz(E_int(P, n1, n2, type, type2, S[i + 1], S[j - 1], S[p - 1],
                                           S[q + 1]));
                    }
                }
                /* multiloop closed by (i,j) */
                int tt = RTYPE[type];
                double s = 0.0;
                for (int k = i + 2; k <= j - 1; k++) {
                    s += qm[IDX(i + 1, k - 1)] * qm1[IDX(k, j - 1)];
                    cm++;
                }
                qbt += s * boltz(P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]));
                if (motif_at(m, i, j)) qbt += m->m_extra;
                qb[IDX(i, j)] = qbt;
                T->stemM[IDX(i, j)] = boltz(E_ml_stem(P, type, S[i - 1], S[j + 1]));
            }
            /* qm1 */
            double v = qb[IDX(i, j)] * T->stemM[IDX(i, j)];
            if (up[j] >= 1) v += qm1[IDX(i, j - 1)] * eMLbase;
            qm1[IDX(i, j)] = v;
            /* qm */
            double w = 0.0, pw = 1.0;
            for (int k = i; k <= j; k++) {
                double pre = (k == i || up[i] >= k - i) ? pw : 0.0;
                if (k > i) pre += qm[IDX(i, k - 1)];
                w += pre * qm1[IDX(k, j)];
                pw *= eMLbase;
                cm++;
            }
            qm[IDX(i, j)] = w;
        }
    }
    double *q5 = T->q5;
    q5[0] = 1.0;
    for (int j = 1; j <= N; j++) {
        double v = (up[j] >= 1) ? q5[j - 1] : 0.0;
        for (int k = 1; k + ORC_TURN + 1 <= j; k++) {
            if (qb[IDX(k, j)] == 0.0) continue;
            int type = PAIR[S[k]][S[j]];
            v += q5[k - 1] * qb[IDX(k, j)] *
                 boltz(E_ext_stem(P, type, k > 1 ? S[k - 1] : -1, j < N ? S[j + 1] : -1));
        }
        q5[j] = v;
    }
    if (nint) *nint = ci;
    if (nml) *nml = cm;
    return q5[N];
}

static void pf_free(pf_tables *T) {
    free(T->qb); free(T->qm); free(T->qm1); free(T->q5); free(T->stemM);
}

static double energy_from_Z(double Z) {
    if (!(Z > 0.0)) return INFINITY;
    return -log(Z) * orc_kT_cal() / 1000.0;
}

double orc_pf_energy_counted(const orc_params *P, const char *seq, const char *constraint,
                             const orc_motif *motif, int64_t *n_int, int64_t *n_ml) {
    model_t m;
    if (!model_init(&m, P, seq, constraint, motif)) {
        model_free(&m);
        return NAN;
    }
    pf_tables T;
    double Z = pf_inside(&m, &T, n_int, n_ml);
    pf_free(&T);
    model_free(&m);
    return energy_from_Z(Z);
}

double orc_pf_energy(const orc_params *P, const char *seq, const char *constraint,
                     const orc_motif *motif) {
    return orc_pf_energy_counted(P, seq, constraint, motif, NULL, NULL);
}

/* ------------------------------------------------------ outside / bppm */
/* Reverse-mode (adjoint) sweep over the inside recursions: for an
 * unambiguous decomposition Z is linear in each qb[i][j], so
 * P(i,j) = qb[i][j] * dZ/dqb[i][j] / Z (McCaskill's outside quantity). */
double orc_bppm(const orc_params *P, const char *seq, const char *constraint,
                const orc_motif *motif, double *probs) {
    model_t m;
    int N0 = (int)strlen(seq);
    if (!model_init(&m, P, seq, constraint, motif)) {
        model_free(&m);
        return NAN;
    }
    pf_tables T;
    double Z = pf_inside(&m, &T, NULL, NULL);
    const int N = m.N;
    const int *S = m.S;
    const int *up = m.hc.up;
    size_t sz = (size_t)(N + 2) * (N + 2);
    double *qbb = (double *)calloc(sz, sizeof(double));
    double *qmb = (double *)calloc(sz, sizeof(double));
    double *qm1b = (double *)calloc(sz, sizeof(double));
    double *q5b = (double *)calloc(N + 2, sizeof(double));
    double eMLbase = boltz(P->MLbase);
    for (int k = 0; k < N0 * N0; k++) probs[k] = 0.0;
    if (Z > 0.0) {
        q5b[N] = 1.0;
        for (int j = N; j >= 1; j--) {
            if (up[j] >= 1) q5b[j - 1] += q5b[j];
            for (int k = 1; k + ORC_TURN + 1 <= j; k++) {
                double qbkj = T.qb[IDX(k, j)];
                if (qbkj == 0.0) continue;
                int type = PAIR[S[k]][S[j]];
                double ext = boltz(E_ext_stem(P, type, k > 1 ? S[k - 1] : -1, j < N ? S[j + 1] : -1));
                q5b[k - 1] += q5b[j] * qbkj * ext;
                qbb[IDX(k, j)] += q5b[j] * T.q5[k - 1] * ext;
            }
        }
        for (int d = N - 1; d >= ORC_TURN + 1; d--) {
            for (int i = 1; i + d <= N; i++) {
                int j = i + d;
                /* qm */
                double g = qmb[IDX(i, j)];
                if (g != 0.0) {
                    double pw = 1.0;
                    for (int k = i; k <= j; k++) {
                        double pre = (k == i || up[i] >= k - i) ? pw : 0.0;
                        if (k > i) {
                            pre += T.qm[IDX(i, k - 1)];
                            qmb[IDX(i, k - 1)] += g * T.qm1[IDX(k, j)];
                        }
                        qm1b[IDX(k, j)] += g * pre;
                        pw *= eMLbase;
                    }
                }
                /* qm1 */
                g = qm1b[IDX(i, j)];
                if (g != 0.0) {
                    qbb[IDX(i, j)] += g * T.stemM[IDX(i, j)];
                    if (up[j] >= 1) qm1b[IDX(i, j - 1)] += g * eMLbase;
                }
                /* qb */
                g = qbb[IDX(i, j)];
                if (g != 0.0 && can_pair(&m, i, j)) {
                    int type = PAIR[S[i]][S[j]];
                    for (int p = i + 1; p <= i + ORC_MAXLOOP + 1 && p < j - ORC_TURN - 1; p++) {
                        int n1 = p - i - 1;
                        if (n1 > 0 && up[i + 1] < n1) break;
                        int minq = j - 1 - (ORC_MAXLOOP - n1);
                        if (minq < p + ORC_TURN + 1) minq = p + ORC_TURN + 1;
                        for (int q = j - 1; q >= minq; q--) {
                            int n2 = j - q - 1;
                            if (n2 > 0 && up[q + 1] < n2) break;
                            if (!can_pair(&m, p, q)) continue;
                            int type2 = PAIR[S[q]][S[p]];
                            qbb[IDX(p, q)] += g * boltz(E_int(P, n1, n2, type, type2, S[i + 1],
                                                              S[j - 1], S[p - 1], S[q + 1]));
                        }
                    }
                    int tt = RTYPE[type];
                    double f = g * boltz(P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]));
                    for (int k = i + 2; k <= j - 1; k++) {
                        qmb[IDX(i + 1, k - 1)] += f * T.qm1[IDX(k, j - 1)];
                        qm1b[IDX(k, j - 1)] += f * T.qm[IDX(i + 1, k - 1)];
                    }
                    if (motif_at(&m, i, j)) {
                        /* the motif's inner pairs carry the extra weight too */
                        double pm = g * m.m_extra / Z;
                        for (int k = 1; k < m.mL - 1; k++) {
                            int pk = m.mpt[k];
                            if (pk > k) {
                                probs[(i + k - 1) * N0 + (i + pk - 1)] += pm;
                                probs[(i + pk - 1) * N0 + (i + k - 1)] += pm;
                            }
                        }
                    }
                }
            }
        }
        for (int i = 1; i <= N; i++)
            for (int j = i + ORC_TURN + 1; j <= N; j++) {
                double p = T.qb[IDX(i, j)] * qbb[IDX(i, j)] / Z;
                probs[(i - 1) * N0 + (j - 1)] += p;
                probs[(j - 1) * N0 + (i - 1)] += p;
            }
    }
    free(qbb); free(qmb); free(qm1b); free(q5b);
    pf_free(&T);
    model_free(&m);
    return energy_from_Z(Z);
}

/* ------------------------------------------------------ structure eval */
double orc_eval_structure(const orc_params *P, const char *seq, const char *structure) {
    int N = (int)strlen(seq);
    if ((int)strlen(structure) != N) return NAN;
    int *S = (int *)malloc(sizeof(int) * (N + 2));
    char *useq = (char *)malloc(N + 2);
    int *pt = (int *)calloc(N + 2, sizeof(int));
    int *stk = (int *)malloc(sizeof(int) * (N + 2)), sp = 0;
    useq[0] = ' ';
    for (int i = 1; i <= N; i++) {
        S[i] = enc_base(seq[i - 1]);
        char c = seq[i - 1];
        if (c >= 'a' && c <= 'z') c = (char)(c - 32);
        if (c == 'T') c = 'U';
        useq[i] = c;
    }
    useq[N + 1] = 0;
    S[0] = S[N];
    S[N + 1] = S[1];
    double e = 0.0;
    int bad = 0;
    for (int i = 1; i <= N; i++) {
        if (structure[i - 1] == '(') stk[sp++] = i;
        else if (structure[i - 1] == ')') {
            if (!sp) { bad = 1; break; }
            int a = stk[--sp];
            pt[a] = i;
            pt[i] = a;
        }
    }
    if (sp) bad = 1;
    if (!bad) {
        /* exterior loop */
        for (int i = 1; i <= N; i++) {
            if (pt[i] > i) {
                int j = pt[i];
                e += E_ext_stem(P, PAIR[S[i]][S[j]], i > 1 ? S[i - 1] : -1, j < N ? S[j + 1] : -1);
                i = j;
            }
        }
        for (int i = 1; i <= N; i++) {
            int j = pt[i];
            if (j <= i) continue;
            int type = PAIR[S[i]][S[j]];
            if (!type) { bad = 1; break; }
            /* enumerate branches inside (i,j) */
            int nb = 0, p = 0, q = 0, unp = 0;
            double ml = 0.0;
            for (int k = i + 1; k < j; k++) {
                if (pt[k] > k) {
                    nb++;
                    if (nb == 1) { p = k; q = pt[k]; }
                    ml += E_ml_stem(P, PAIR[S[k]][S[pt[k]]], S[k - 1], S[pt[k] + 1]);
                    k = pt[k];
                } else unp++;
            }
            if (nb == 0) e += E_hairpin(P, i, j, S, useq);
            else if (nb == 1) {
                int type2 = PAIR[S[q]][S[p]];
                if (!type2) { bad = 1; break; }
                e += E_int(P, p - i - 1, j - q - 1, type, type2, S[i + 1], S[j - 1], S[p - 1], S[q + 1]);
            } else {
                e += P->MLclosing + E_ml_stem(P, RTYPE[type], S[j - 1], S[i + 1]) + ml +
                     unp * P->MLbase;
            }
        }
    }
    free(S); free(useq); free(pt); free(stk);
    return bad ? NAN : e / 100.0;
}

/* ---------------------------------------------------------------- MFE */
#define MINF 100000000
static int min2(int a, int b) { return a < b ? a : b; }

static int E_hairpin_int(const orc_params *P, int i, int j, const int *S, const char *useq) {
    int u = j - i - 1;
    int type = PAIR[S[i]][S[j]];
    int e = (u <= 30) ? P->hairpin[u] : P->hairpin[30] + (int)(P->lxc * log(u / 30.0));
    if (u < 3) return e;
    if (u == 4) {
        for (int k = 0; k < P->ntetra; k++)
            if (strncmp(useq + i, P->tetra[k], 6) == 0) return P->tetraE[k];
    } else if (u == 6) {
        for (int k = 0; k < P->nhexa; k++)
            if (strncmp(useq + i, P->hexa[k], 8) == 0) return P->hexaE[k];
    } else if (u == 3) {
        for (int k = 0; k < P->ntri; k++)
            if (strncmp(useq + i, P->tri[k], 5) == 0) return P->triE[k];
        return e + (type > 2 ? P->TermAU : 0);
    }
    return e + P->mmH[type][S[i + 1]][S[j - 1]];
}

int orc_mfe(const orc_params *P, const char *seq, const char *constraint, char *structure) {
    model_t m;
    if (!model_init(&m, P, seq, constraint, NULL)) {
        model_free(&m);
        return MINF;
    }
    const int N = m.N;
    const int *S = m.S;
    const int *up = m.hc.up;
    size_t sz = (size_t)(N + 2) * (N + 2);
    int *c = (int *)malloc(sz * sizeof(int));
    int *fm = (int *)malloc(sz * sizeof(int));
    int *fm1 = (int *)malloc(sz * sizeof(int));
    int *f5 = (int *)malloc((N + 2) * sizeof(int));
    for (size_t k = 0; k < sz; k++) { c[k] = MINF; fm[k] = MINF; fm1[k] = MINF; }
    for (int d = ORC_TURN + 1; d <= N - 1; d++) {
        for (int i = 1; i + d <= N; i++) {
            int j = i + d;
            int best = MINF;
            if (can_pair(&m, i, j)) {
                int type = PAIR[S[i]][S[j]];
                int u = j - i - 1;
                if (up[i + 1] >= u) best = E_hairpin_int(P, i, j, S, m.useq);
                for (int p = i + 1; p <= i + ORC_MAXLOOP + 1 && p < j - ORC_TURN - 1; p++) {
                    int n1 = p - i - 1;
                    if (n1 > 0 && up[i + 1] < n1) break;
                    int minq = j - 1 - (ORC_MAXLOOP - n1);
                    if (minq < p + ORC_TURN + 1) minq = p + ORC_TURN + 1;
                    for (int q = j - 1; q >= minq; q--) {
                        int n2 = j - q - 1;
                        if (n2 > 0 && up[q + 1] < n2) break;
                        if (!can_pair(&m, p, q) || c[IDX(p, q)] >= MINF) continue;
                        int type2 = PAIR[S[q]][S[p]];
                        int e = (int)E_int(P, n1, n2, type, type2, S[i + 1], S[j - 1], S[p - 1], S[q + 1]);
                        best = min2(best, c[IDX(p, q)] + e);
                    }
                }
                int tt = RTYPE[type];
                int s = MINF;
                for (int k = i + 2; k <= j - 1; k++)
                    if (fm[IDX(i + 1, k - 1)] < MINF && fm1[IDX(k, j - 1)] < MINF)
                        s = min2(s, fm[IDX(i + 1, k - 1)] + fm1[IDX(k, j - 1)]);
                if (s < MINF) best = min2(best, s + P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]));
                c[IDX(i, j)] = best;
            }
            int v = MINF;
            if (c[IDX(i, j)] < MINF)
                v = c[IDX(i, j)] + E_ml_stem(P, PAIR[S[i]][S[j]], S[i - 1], S[j + 1]);
            if (up[j] >= 1 && fm1[IDX(i, j - 1)] < MINF) v = min2(v, fm1[IDX(i, j - 1)] + P->MLbase);
            fm1[IDX(i, j)] = v;
            int w = MINF;
            for (int k = i; k <= j; k++) {
                if (fm1[IDX(k, j)] >= MINF) continue;
                int pre = MINF;
                if (k == i || up[i] >= k - i) pre = (k - i) * P->MLbase;
                if (k > i && fm[IDX(i, k - 1)] < MINF) pre = min2(pre, fm[IDX(i, k - 1)]);
                if (pre < MINF) w = min2(w, pre + fm1[IDX(k, j)]);
            }
            fm[IDX(i, j)] = w;
        }
    }
    f5[0] = 0;
    for (int j = 1; j <= N; j++) {
        int v = (up[j] >= 1 && f5[j - 1] < MINF) ? f5[j - 1] : MINF;
        for (int k = 1; k + ORC_TURN + 1 <= j; k++) {
            if (c[IDX(k, j)] >= MINF || f5[k - 1] >= MINF) continue;
            int type = PAIR[S[k]][S[j]];
            v = min2(v, f5[k - 1] + c[IDX(k, j)] +
                            E_ext_stem(P, type, k > 1 ? S[k - 1] : -1, j < N ? S[j + 1] : -1));
        }
        f5[j] = v;
    }
    int result = f5[N];
    if (structure) {
        for (int k = 0; k < N; k++) structure[k] = '.';
        structure[N] = 0;
        if (result < MINF) {
            /* iterative traceback: stack of (kind, i, j); kind 0 = f5 prefix j,
             * 1 = c(i,j), 2 = fm(i,j), 3 = fm1(i,j) */
            int *st = (int *)malloc(sizeof(int) * 3 * (4 * N + 8)), top = 0;
            st[top++] = 0; st[top++] = 0; st[top++] = N;
            while (top) {
                int j = st[--top], i = st[--top], kind = st[--top];
                if (kind == 0) {
                    if (j <= 0) continue;
                    if (up[j] >= 1 && f5[j - 1] == f5[j]) {
                        st[top++] = 0; st[top++] = 0; st[top++] = j - 1;
                        continue;
                    }
                    for (int k = 1; k + ORC_TURN + 1 <= j; k++) {
                        if (c[IDX(k, j)] >= MINF || f5[k - 1] >= MINF) continue;
                        int type = PAIR[S[k]][S[j]];
                        if (f5[k - 1] + c[IDX(k, j)] +
                                E_ext_stem(P, type, k > 1 ? S[k - 1] : -1, j < N ? S[j + 1] : -1) == f5[j]) {
                            st[top++] = 0; st[top++] = 0; st[top++] = k - 1;
                            st[top++] = 1; st[top++] = k; st[top++] = j;
                            break;
                        }
                    }
                } else if (kind == 1) {
                    structure[i - 1] = '(';
                    structure[j - 1] = ')';
                    int type = PAIR[S[i]][S[j]];
                    int target = c[IDX(i, j)];
                    int u = j - i - 1;
                    if (up[i + 1] >= u && E_hairpin_int(P, i, j, S, m.useq) == target) continue;
                    int found = 0;
                    for (int p = i + 1; !found && p <= i + ORC_MAXLOOP + 1 && p < j - ORC_TURN - 1; p++) {
                        int n1 = p - i - 1;
                        if (n1 > 0 && up[i + 1] < n1) break;
                        int minq = j - 1 - (ORC_MAXLOOP - n1);
                        if (minq < p + ORC_TURN + 1) minq = p + ORC_TURN + 1;
                        for (int q = j - 1; q >= minq; q--) {
                            int n2 = j - q - 1;
                            if (n2 > 0 && up[q + 1] < n2) break;
                            if (!can_pair(&m, p, q) || c[IDX(p, q)] >= MINF) continue;
                            int type2 = PAIR[S[q]][S[p]];
                            int e = (int)E_int(P, n1, n2, type, type2, S[i + 1], S[j - 1], S[p - 1], S[q + 1]);
                            if (c[IDX(p, q)] + e == target) {
                                st[top++] = 1; st[top++] = p; st[top++] = q;
                                found = 1;
                                break;
                            }
                        }
                    }
                    if (found) continue;
                    int tt = RTYPE[type];
                    int cl = P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]);
                    for (int k = i + 2; k <= j - 1; k++) {
                        if (fm[IDX(i + 1, k - 1)] < MINF && fm1[IDX(k, j - 1)] < MINF &&
                            fm[IDX(i + 1, k - 1)] + fm1[IDX(k, j - 1)] + cl == target) {
                            st[top++] = 2; st[top++] = i + 1; st[top++] = k - 1;
                            st[top++] = 3; st[top++] = k; st[top++] = j - 1;
                            break;
                        }
                    }
                } else if (kind == 3) {
                    int target = fm1[IDX(i, j)];
                    if (c[IDX(i, j)] < MINF &&
                        c[IDX(i, j)] + E_ml_stem(P, PAIR[S[i]][S[j]], S[i - 1], S[j + 1]) == target) {
                        st[top++] = 1; st[top++] = i; st[top++] = j;
                    } else {
                        st[top++] = 3; st[top++] = i; st[top++] = j - 1;
                    }
                } else {
                    int target = fm[IDX(i, j)];
                    for (int k = i; k <= j; k++) {
                        if (fm1[IDX(k, j)] >= MINF) continue;
                        if ((k == i || up[i] >= k - i) && (k - i) * P->MLbase + fm1[IDX(k, j)] == target) {
                            st[top++] = 3; st[top++] = k; st[top++] = j;
                            break;
                        }
                        if (k > i && fm[IDX(i, k - 1)] < MINF && fm[IDX(i, k - 1)] + fm1[IDX(k, j)] == target) {
                            st[top++] = 2; st[top++] = i; st[top++] = k - 1;
                            st[top++] = 3; st[top++] = k; st[top++] = j;
                            break;
                        }
                    }
                }
            }
            free(st);
        }
    }
    free(c); free(fm); free(fm1); free(f5);
    model_free(&m);
    return result;
}

/* ------------------------------------------------- MFE with the motif */
/* Minimum free energy (kcal/mol) of the same model the partition function
 * sums over, for the engine's MFE fold mode: the min-plus
 * form of the inside recursion of orc_mfe above, integer dcal/mol throughout
 * (held in doubles, every value integral), with the ligand motif entering like
 * it does in the partition function -- a formed motif's closing cell may take
 * the motif structure's energy plus the bonus, rounded once to dcal:
 * c(i,j) = min(c(i,j), lround(100*(Eint + bonus))) (the min-plus image of the
 * extra term exp(-Eint)(exp(-bonus) - 1) the PF adds at the same cell). */
double orc_mfe_energy(const orc_params *P, const char *seq, const char *constraint,
                      const orc_motif *motif) {
    model_t m;
    if (!model_init(&m, P, seq, constraint, motif)) {
        model_free(&m);
        return NAN;
    }
    const int N = m.N;
    const int *S = m.S;
    const int *up = m.hc.up;
    const double INF = 1e30;
    size_t sz = (size_t)(N + 2) * (N + 2);
    double *c = (double *)malloc(sz * sizeof(double));
    double *fm = (double *)malloc(sz * sizeof(double));
    double *fm1 = (double *)malloc(sz * sizeof(double));
    double *f5 = (double *)malloc((N + 2) * sizeof(double));
    for (size_t k = 0; k < sz; k++) { c[k] = INF; fm[k] = INF; fm1[k] = INF; }
    for (int d = ORC_TURN + 1; d <= N - 1; d++) {
        for (int i = 1; i + d <= N; i++) {
            int j = i + d;
            double best = INF;
            if (can_pair(&m, i, j)) {
                int type = PAIR[S[i]][S[j]];
                int u = j - i - 1;
                if (up[i + 1] >= u) best = E_hairpin_int(P, i, j, S, m.useq);
                for (int p = i + 1; p <= i + ORC_MAXLOOP + 1 && p < j - ORC_TURN - 1; p++) {
                    int n1 = p - i - 1;
                    if (n1 > 0 && up[i + 1] < n1) break;
                    int minq = j - 1 - (ORC_MAXLOOP - n1);
                    if (minq < p + ORC_TURN + 1) minq = p + ORC_TURN + 1;
                    for (int q = j - 1; q >= minq; q--) {
                        int n2 = j - q - 1;
                        if (n2 > 0 && up[q + 1] < n2) break;
                        if (!can_pair(&m, p, q) || c[IDX(p, q)] >= INF) continue;
                        int type2 = PAIR[S[q]][S[p]];
                        double e = (int)E_int(P, n1, n2, type, type2, S[i + 1], S[j - 1], S[p - 1], S[q + 1]);
                        if (c[IDX(p, q)] + e < best) best = c[IDX(p, q)] + e;
                    }
                }
                int tt = RTYPE[type];
                double sm = INF;
                for (int k = i + 2; k <= j - 1; k++)
                    if (fm[IDX(i + 1, k - 1)] < INF && fm1[IDX(k, j - 1)] < INF &&
                        fm[IDX(i + 1, k - 1)] + fm1[IDX(k, j - 1)] < sm)
                        sm = fm[IDX(i + 1, k - 1)] + fm1[IDX(k, j - 1)];
                if (sm < INF && sm + P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]) < best)
                    best = sm + P->MLclosing + E_ml_stem(P, tt, S[j - 1], S[i + 1]);
                if (m.mL && motif_at(&m, i, j)) {
                    if (m.m_mfe_dcal < best) best = m.m_mfe_dcal;
                }
                c[IDX(i, j)] = best;
            }
            double v = INF;
            if (c[IDX(i, j)] < INF) v = c[IDX(i, j)] + E_ml_stem(P, PAIR[S[i]][S[j]], S[i - 1], S[j + 1]);
            if (up[j] >= 1 && fm1[IDX(i, j - 1)] < INF && fm1[IDX(i, j - 1)] + P->MLbase < v)
                v = fm1[IDX(i, j - 1)] + P->MLbase;
            fm1[IDX(i, j)] = v;
            double w = INF;
            for (int k = i; k <= j; k++) {
                if (fm1[IDX(k, j)] >= INF) continue;
                double pre = INF;
                if (k == i || up[i] >= k - i) pre = (double)(k - i) * P->MLbase;
                if (k > i && fm[IDX(i, k - 1)] < pre) pre = fm[IDX(i, k - 1)];
                if (pre < INF && pre + fm1[IDX(k, j)] < w) w = pre + fm1[IDX(k, j)];
            }
            fm[IDX(i, j)] = w;
        }
    }
    f5[0] = 0.0;
    for (int j = 1; j <= N; j++) {
        double v = (up[j] >= 1 && f5[j - 1] < INF) ? f5[j - 1] : INF;
        for (int k = 1; k + ORC_TURN + 1 <= j; k++) {
            if (c[IDX(k, j)] >= INF || f5[k - 1] >= INF) continue;
            int type = PAIR[S[k]][S[j]];
            double e = f5[k - 1] + c[IDX(k, j)] + E_ext_stem(P, type, k > 1 ? S[k - 1] : -1, j < N ? S[j + 1] : -1);
            if (e < v) v = e;
        }
        f5[j] = v;
    }
    double r = f5[N] >= INF ? INFINITY : f5[N] / 100.0;
    free(c); free(fm); free(fm1); free(f5);
    model_free(&m);
    return r;
}
