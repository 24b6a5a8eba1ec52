/*
 * adx_oracle.h -- CPU restatement of addapt's fold -> score -> accept hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in addapt_amd/ (the product) may link,
 * import or execute this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * What it restates (reference = /root/reference, read-only):
 *   - the ViennaRNA-2.x McCaskill inside partition function that
 *     ViennaRnaFold::macrostate_prob drives (src/scoring.cc:53-71, 73-103):
 *     default model (37 C, dangles=2, TURN=3, MAXLOOP=30, special hairpins),
 *     dot-bracket hard constraints with ENFORCE_BP (scoring.cc:61-62) and the
 *     ligand hairpin/interior motif soft constraint (scoring.cc:92-100);
 *     unscaled double precision, plain O(N^3)/O(N^2 L^2) loops;
 *   - MacrostateProbTerm / ScoreFunction (scoring.cc:114-158, 233-259);
 *   - MonteCarlo::apply (src/sampling.cc:22-107) with the three RNG streams,
 *     UnbiasedMutationMove (sampling.cc:287-303), mutate_recursively
 *     (sampling.cc:195-282), the three thermostats (sampling.cc:305-401) and the
 *     Metropolis test (sampling.cc:76-89);
 *   - std::mt19937, libstdc++-11 uniform_int_distribution (Lemire) and
 *     generate_canonical<double,53> (the streams addapt draws from).
 *
 * Parity pins (see DESIGN.md "Parity"): the reference cannot be built here
 * (ViennaRNA, boost, yaml-cpp and docopt are absent), so this oracle is pinned
 * by the reference's own known-answer tests (tests/test_sampling.cc,
 * tests/test_model.cc, tests/test_scoring.cc:261-384), by its threshold tests
 * and RNAfold annotations (test_scoring.cc:52-55, 83-259), by libstdc++ RNG
 * golden values, and by an independent exhaustive-enumeration checker for short
 * sequences (tests/test_oracle_enum.py).  Exact ViennaRNA energy values are
 * "parity unpinned": the parameter VALUES are authored offline.
 */
#ifndef ADX_ORACLE_H
#define ADX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_INF 10000000
#define ORC_MAXLOOP 30
#define ORC_TURN 3

typedef struct orc_params {
    int stack[8][8];
    int mmH[8][5][5], mmI[8][5][5], mm1nI[8][5][5], mm23I[8][5][5];
    int mmM[8][5][5], mmExt[8][5][5];
    int d5[8][5], d3[8][5];
    int int11[8][8][5][5];
    int int21[8][8][5][5][5];
    int int22[8][8][5][5][5][5];
    int hairpin[31], bulge[31], interior[31];
    int MLbase, MLclosing, MLintern;
    int ninio, maxninio, TermAU, DuplexInit;
    double lxc;
    int ntri, ntetra, nhexa;
    char tri[32][8];
    char tetra[64][8];
    char hexa[32][12];
    int triE[32], tetraE[64], hexaE[32];
} orc_params;

/* kT at 37 C in cal/mol (ViennaRNA: (T + K0) * GASCONST). */
double orc_kT_cal(void);

/* ---- parameters ------------------------------------------------------- */
/* Parse a ViennaRNA 2.0 parameter file; returns NULL and sets the error
 * message (orc_last_error) on failure.  Caller frees with orc_params_free. */
orc_params *orc_params_load(const char *path);
void orc_params_free(orc_params *P);
const char *orc_last_error(void);

/* ---- folding ---------------------------------------------------------- */
/* Ligand motif (vrna_sc_add_hi_motif, scoring.cc:92-100).  mode 0 = "auto"
 * (the default: add in partition functions, replace in the MFE -- the
 * conventions the reference's RNAfold annotations pin, test_scoring.cc:52-55
 * and :154), mode 1 = "add" (bonus added to the motif structure's intrinsic
 * energy), mode 2 = "replace" (motif structure's total energy := bonus);
 * the numbering of the engine's ADX_MOTIF_*. */
typedef struct orc_motif {
    const char *seq;     /* upper case ACGU */
    const char *fold;    /* dot-bracket, outer pair spans the motif */
    double energy_kcal;  /* kT*ln(Kd/1M) in the reference */
    int mode;
} orc_motif;

/* Ensemble free energy (kcal/mol, double; the caller rounds to float to
 * mimic vrna_pf's float return).  seq: N chars ACGUN (case-insensitive,
 * upper-cased internally as scoring.cc:28 does).  constraint: NULL or an N-char
 * dot-bracket hard constraint applied with DB_DEFAULT|ENFORCE_BP.  motif:
 * NULL for apo.  Returns +inf if the constrained ensemble is empty. */
double orc_pf_energy(const orc_params *P, const char *seq, const char *constraint,
                     const orc_motif *motif);

/* Same, also returning the number of interior-loop / multiloop terms
 * evaluated (for the FLOP accounting in bench.py / DESIGN.md). */
double orc_pf_energy_counted(const orc_params *P, const char *seq, const char *constraint,
                             const orc_motif *motif, int64_t *n_int_terms,
                             int64_t *n_ml_terms);

/* Base-pair probability matrix (inside + outside), dense N*N row-major
 * (0-based, symmetric, zero diagonal).  Returns the ensemble energy. */
double orc_bppm(const orc_params *P, const char *seq, const char *constraint,
                const orc_motif *motif, double *probs);

/* Free energy (kcal/mol) of one structure: loop decomposition with the same
 * model (dangles=2, PF-style non-truncated lxc), no motif bonus. */
double orc_eval_structure(const orc_params *P, const char *seq, const char *structure);

/* Minimum free energy (integer dcal/mol, lxc truncated as in ViennaRNA's MFE
 * recursions); writes the MFE structure if structure != NULL (N+1 bytes). */
int orc_mfe(const orc_params *P, const char *seq, const char *constraint, char *structure);
/* MFE (kcal/mol) with the ligand motif, min-plus image of the PF model (fold.c) */
double orc_mfe_energy(const orc_params *P, const char *seq, const char *constraint, const orc_motif *motif);

/* ---- RNG -------------------------------------------------------------- */
typedef struct orc_mt {
    uint32_t mt[624];
    int idx;
} orc_mt;

void orc_mt_seed(orc_mt *g, uint32_t seed);
uint32_t orc_mt_next(orc_mt *g);
/* std::uniform_int_distribution<int>(a, b)(g) as in libstdc++ >= 11 */
int orc_uniform_int(orc_mt *g, int a, int b);
/* std::uniform_real_distribution<double>(0,1)(g) = generate_canonical<double,53> */
double orc_canonical(orc_mt *g);
/* std::nth_element (libstdc++ 11 introselect, step for step) and the
 * std::max(t, 0.0) clamp of AutoScalingThermostat (sampling.cc:389-396). */
void orc_nth_element(double *a, long k, long n);
double orc_auto_clamp(double t);

/* ---- mutation move ---------------------------------------------------- */
/* Device = sequence + M macrostates (each N chars).  Error codes: */
#define ORC_MUT_OK 0
#define ORC_MUT_MISMATCHED_BRACKET 1
#define ORC_MUT_IMMUTABLE_PARTNER 2
#define ORC_MUT_UNSATISFIABLE 3

int orc_can_be_mutated(const char *seq, int pos);
int orc_can_be_freely_mutated(const char *seq, int n, const char *const *macrostates,
                              int n_macro, int pos);
/* mutate_recursively (sampling.cc:195-282); seq is modified in place. */
int orc_mutate_recursively(char *seq, int n, const char *const *macrostates, int n_macro,
                           int pos, char base);

/* ---- score function + Monte Carlo ------------------------------------- */
typedef struct orc_term {
    int condition;  /* 0 = apo, 1 = holo */
    int macrostate; /* index into the macrostate list (kind 0) */
    int favorable;  /* 1 = YES, 0 = NO ("not <name>") */
    double weight;
    int kind;       /* 0 = MacrostateProbTerm (scoring.cc:233-259); 1 = base-pair
                       probability term: p = RnaFold::base_pair_prob(i, j) of the
                       condition's unconstrained fold (scoring.cc:37-51) */
    int pair_i, pair_j; /* kind 1: 0-based device positions (context-shifted) */
} orc_term;

typedef struct orc_context {
    const char *before;
    const char *after;
} orc_context;

typedef struct orc_scorefxn {
    const orc_params *P;
    int n_terms;
    const orc_term *terms;
    const orc_motif *aptamer; /* NULL = no aptamer: holo folds like apo */
    int n_contexts;           /* 0 = no contexts; else in std::map (name) order */
    const orc_context *contexts;
    int mode;                 /* 0 = partition functions (vrna_pf), 1 = MFE (A17) */
} orc_scorefxn;

/* ScoreFunction::evaluate; term_values (n_terms * max(1,n_contexts)) and
 * dG (2 * (1 + n_macro_used) per context...) are optional outputs:
 * term_values[c*n_terms + t].  Returns the score. */
double orc_score(const orc_scorefxn *sf, const char *seq, int n, const char *const *macrostates,
                 int n_macro, double *term_values);

typedef struct orc_thermostat {
    int kind; /* 0 fixed, 1 annealing, 2 auto-scaling */
    double t_fixed;
    double t_hi, t_lo;
    int cycle_len;
    double target_rate;
    int period;
    double t_init;
} orc_thermostat;

/* Outcomes (sampling.hh:88-93) */
#define ORC_REJECT 0
#define ORC_ACCEPT_WORSENED 1
#define ORC_ACCEPT_UNCHANGED 2
#define ORC_ACCEPT_IMPROVED 3

/* Per-step trace (optional arrays of length num_steps). */
typedef struct orc_trace {
    int *pos;             /* chosen position (freely-mutable list entry) */
    char *base;           /* chosen base */
    int *outcome;
    double *temperature;
    double *proposed_score; /* NAN on unchanged steps */
    double *current_score;  /* after the step */
    double *random_threshold;
    char *seqs;           /* num_steps * n current sequence after the step, or NULL */
} orc_trace;

/* Callback used to resolve near-tie Metropolis decisions during GPU parity
 * replay: if non-NULL and |crit - u| <= tie_eps, *forced* decides. */
typedef struct orc_mc_opts {
    double tie_eps;
    const int *forced_outcome; /* per step, or NULL */
} orc_mc_opts;

/* MonteCarlo::apply for one walker.  seq (n chars) is updated in place to the
 * final current sequence; counters[4] receives the outcome counts.  Returns
 * ORC_MUT_* error from the move (0 on success). */
int orc_mc_run(const orc_scorefxn *sf, char *seq, int n, const char *const *macrostates,
               int n_macro, const orc_thermostat *th, uint32_t seed, int num_steps,
               double *final_score, int64_t *counters, orc_trace *trace,
               const orc_mc_opts *opts);

/* CPU baseline: W independent walkers over n_threads OpenMP threads, each
 * walker w running orc_mc_run from seqs[w*n] with seed seeds[w].  Returns the
 * wall time in seconds. */
double orc_mc_run_batch(const orc_scorefxn *sf, char *seqs, int n, int W,
                        const char *const *macrostates, int n_macro,
                        const orc_thermostat *th, const uint32_t *seeds, int num_steps,
                        int n_threads, int64_t *counters_total);

#ifdef __cplusplus
}
#endif
#endif
