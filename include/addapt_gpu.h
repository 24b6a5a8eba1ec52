/*
 * addapt_gpu.h -- C ABI of the MI355X (gfx950) fold -> score -> accept engine.
 *
 * Plain C, plain pointers and sizes, status codes, no exceptions, no torch
 * types.  Library: addapt_amd/_lib/libaddapt_gpu.so (built by
 * __graft_entry__.build()).  All calls are synchronous; one context per GPU
 * per host thread; calls on one context must be serialised by the caller.
 *
 * Two layers, both replacing the reference's FFI into ViennaRNA
 * (/root/reference/src/scoring.cc:6-11 includes, 37-103 call sites):
 *
 *  (1) the per-fold layer adx_fold_* -- one entry point per ViennaRNA symbol
 *      the reference binds, for code that keeps addapt's RnaFold interface
 *      (scoring.hh:42-55, ViennaRnaFold scoring.cc:17-103);
 *
 *  (2) the batched Monte Carlo layer adx_ctx_* / adx_walkers_* / adx_run_steps
 *      / adx_score_batch -- thousands of independent walkers in lockstep;
 *      each step of MonteCarlo::apply (sampling.cc:55-99) is three launches
 *      on one stream, no host round trip: propose (move + thermostat + RNG),
 *      fold + score of the changed walkers, Metropolis accept (plus the
 *      outside pass when base-pair terms are scored).
 */
#ifndef ADDAPT_GPU_H
#define ADDAPT_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADX_ABI_VERSION 4

typedef enum adx_status {
    ADX_OK = 0,
    ADX_EINVAL = 1,      /* bad argument / malformed input */
    ADX_EHIP = 2,        /* HIP runtime error */
    ADX_ECONSTRAINT = 3, /* malformed dot-bracket constraint */
    ADX_EPARAM = 4,      /* energy-parameter file could not be read */
    ADX_ENOMEM = 5,      /* allocation failed */
    ADX_EMOVE = 6,       /* mutation move failed (sampling.cc:256,265,279) */
    ADX_ESTATE = 7,      /* call out of order (e.g. run before walkers_init) */
    ADX_ENODEV = 8,      /* no gfx950 device visible */
    ADX_EUNSUPPORTED = 9 /* feature not available on the GPU path */
} adx_status;

/* Thread-local message for the last non-OK status. */
const char *adx_last_error(void);
int adx_abi_version(void);

/* ------------------------------------------------------------------------
 * Energy parameters (ViennaRNA 2.0 parameter-file layout).  Replaces the
 * implicit vrna_md_set_default() model (scoring.cc:80-83): 37 C, dangles=2,
 * special hairpins, TURN=3, MAXLOOP=30.
 * ---------------------------------------------------------------------- */
typedef struct adx_params adx_params;
adx_status adx_params_load(const char *par_path, adx_params **out);
void adx_params_free(adx_params *p);
/* kT at 37 C in kcal/mol (= fc->exp_params->kT / 1000, scoring.cc:69,91). */
double adx_kT(void);
/* Free energy (kcal/mol) of one structure under the loaded model. */
adx_status adx_eval_structure(const adx_params *p, const char *seq, const char *structure,
                              double *energy_kcal);

/* ------------------------------------------------------------------------
 * (1) Per-fold layer: one-to-one with the ViennaRNA calls in scoring.cc.
 * ---------------------------------------------------------------------- */
typedef struct adx_fold adx_fold;
/* vrna_md_set_default + vrna_fold_compound(seq, &md, VRNA_OPTION_PF)
 * (scoring.cc:79-88); with_bppm mirrors md.compute_bpp (scoring.cc:82-83).
 * The sequence is upper-cased as ViennaRnaFold's constructor does (:28). */
adx_status adx_fold_create(const adx_params *p, const char *seq, int with_bppm, int device,
                           adx_fold **out);
/* vrna_sc_add_hi_motif(fc, seq, fold, energy, VRNA_OPTION_DEFAULT) (:92-100) */
adx_status adx_fold_add_motif(adx_fold *f, const char *motif_seq, const char *motif_fold,
                              double energy_kcal);
/* vrna_constraints_add(fc, db, DB_DEFAULT | DB_ENFORCE_BP) (:61-62) */
adx_status adx_fold_add_constraint(adx_fold *f, const char *dot_bracket);
/* vrna_pf(fc, NULL) (:58, :65): ensemble free energy (kcal/mol, float) */
adx_status adx_fold_pf(adx_fold *f, float *energy_kcal);
/* vrna_mfe(fc, NULL) (fold.h, included at scoring.cc:9, never called by the
 * reference): minimum free energy (kcal/mol, float; integer dcal arithmetic;
 * +inf when the constraint admits no structure), with the ligand motif
 * entering as c(i,j) = min(c(i,j), round(100*(E_motif + bonus))) at every site
 * where the motif can form.  Energy only, no structure. */
adx_status adx_fold_mfe(adx_fold *f, float *energy_kcal);
/* fc->exp_matrices->probs[fc->iindx[i] - j] with 1-based i < j (:47-50);
 * computed on first use with md.compute_bpp (:41-44). */
adx_status adx_fold_bpp(adx_fold *f, int i, int j, double *prob);
/* vrna_fold_compound_free (:31-35) */
void adx_fold_free(adx_fold *f);

/* ------------------------------------------------------------------------
 * (2) Batched Monte Carlo layer.
 * ---------------------------------------------------------------------- */
#define ADX_APO 0
#define ADX_HOLO 1

#define ADX_TERM_MACROSTATE 0  /* MacrostateProbTerm (scoring.hh:175-192): p = macrostate_prob */
#define ADX_TERM_PAIR 1        /* p = RnaFold::base_pair_prob(i, j) (scoring.cc:37-51) of the
                                  condition's unconstrained fold (outside pass, configs 3-4) */

typedef struct adx_term {
    int condition;             /* ADX_APO / ADX_HOLO */
    int macrostate;            /* index into adx_run_desc.macrostates (ADX_TERM_MACROSTATE) */
    int favorable;             /* 1 = "<name>" (ln p), 0 = "not <name>" (ln(1 - p)) */
    double weight;             /* ScoreTerm weight (scoring.hh:160-168) */
    int kind;                  /* ADX_TERM_MACROSTATE (zero-initialised default) / ADX_TERM_PAIR */
    int pair_i, pair_j;        /* ADX_TERM_PAIR: 0-based device positions, i < j */
} adx_term;

#define ADX_THERMO_FIXED 0     /* FixedThermostat (sampling.cc:305-321) */
#define ADX_THERMO_ANNEAL 1    /* AnnealingThermostat (:324-378) */
#define ADX_THERMO_AUTO 2      /* AutoScalingThermostat (:381-410) */

typedef struct adx_thermostat {
    int kind;
    double t_fixed;
    double t_hi, t_lo;
    int cycle_len;
    double target_rate;
    int period;
    double t_init;
} adx_thermostat;

#define ADX_MOTIF_AUTO 0       /* default (zero-initialised): ADD in partition functions,
                                  REPLACE in MFE folds -- the convention that holds every
                                  reference pin: the rhf(6) ensemble annotations and holo
                                  classes (test_scoring.cc:54-55) and RNAfold's printed holo
                                  MFE -9.22 (test_scoring.cc:152-154, tools/test_seq:9) */
#define ADX_MOTIF_ADD 1        /* opt-in: ligand bonus added to the motif structure's own loop
                                  energies in both fold modes (holo MFE of THEO: -10.92) */
#define ADX_MOTIF_REPLACE 2    /* opt-in: motif structure's total energy := bonus, both modes */

#define ADX_FOLD_PF 0          /* MacrostateProbTerm over vrna_pf ensembles (scoring.cc:53-71) */
#define ADX_FOLD_MFE 1         /* the same terms over minimum free energies:
                                  p = exp(-(E_mfe(constrained) - E_mfe(free)) / kT) */

typedef struct adx_context_desc { /* Context (model.hh:139-157) */
    const char *before;
    const char *after;
} adx_context_desc;

typedef struct adx_run_desc {
    const adx_params *params;
    const char *sequence;            /* template Device sequence; upper = mutable */
    int n_macrostates;
    const char *const *macrostates;  /* each strlen(sequence) chars */
    int n_terms;
    const adx_term *terms;
    const char *aptamer_seq;         /* NULL: no aptamer (holo folds like apo) */
    const char *aptamer_fold;
    double aptamer_energy_kcal;      /* kT*ln(Kd/1M) (scoring.cc:91-99) */
    int motif_mode;                  /* ADX_MOTIF_AUTO (default, 0) / _ADD / _REPLACE */
    int n_contexts;                  /* 0 = none; else map (name) order */
    const adx_context_desc *contexts;
    adx_thermostat thermostat;
    int device;                      /* HIP device ordinal */
    int fold_mode;                   /* ADX_FOLD_PF (default, zero-initialised) / ADX_FOLD_MFE */
} adx_run_desc;

typedef struct adx_ctx adx_ctx;

typedef struct adx_info {
    int length;          /* N (raw device length) */
    int n_variants;      /* partition functions per scored step */
    int n_terms;         /* score terms per context */
    int n_mutable;       /* freely mutable positions */
    int max_walkers;
    double scale_per_nt; /* pf scaling used by the FP32 kernels */
} adx_info;

adx_status adx_ctx_create(const adx_run_desc *desc, adx_ctx **out);
void adx_ctx_destroy(adx_ctx *ctx);
adx_status adx_ctx_info(const adx_ctx *ctx, adx_info *info);

/* W walkers; seqs = W*N chars (NULL: every walker starts from the template),
 * seeds = W uint32 (std::mt19937(seed) per walker, addapt.cc:89).  Computes
 * the initial score of each walker (sampling.cc:40). */
adx_status adx_walkers_init(adx_ctx *ctx, int n_walkers, const char *seqs,
                            const uint32_t *seeds);

/* Optional per-step trace, host arrays of steps*W entries (step-major). */
typedef struct adx_trace {
    int32_t *position;       /* freely-mutable position chosen */
    char *base;              /* base chosen */
    int32_t *outcome;        /* 0 REJECT 1 WORSENED 2 UNCHANGED 3 IMPROVED */
    double *temperature;
    double *proposed_score;  /* NaN on ACCEPT_UNCHANGED */
    double *current_score;   /* after the step */
    double *random_threshold;
    double *term_values;     /* steps*W*n_terms*max(1,n_contexts), proposed; NaN if unchanged */
} adx_trace;

/* Advance every walker by `steps` MC steps (fused mutate + fold + score +
 * Metropolis); the step counter persists across calls (thermostat index). */
adx_status adx_run_steps(adx_ctx *ctx, int steps, adx_trace *trace);

/* Device time (ms) of the last adx_run_steps / adx_score_batch, measured with
 * HIP events on the context's stream. */
adx_status adx_last_kernel_ms(const adx_ctx *ctx, double *ms);
/* Average duration of the score kernel (the fold -> score launch, the dominant
 * kernel) over the launches of the last adx_run_steps, from HIP events recorded
 * on the context's stream around each launch. */
adx_status adx_last_score_kernel_ms(const adx_ctx *ctx, double *avg_ms, int *launches);
/* The same window split per launch (averages, ms): the inside folds (fold ->
 * energies or scores) and, when score terms read base-pair probabilities, the
 * outside pass on the stored inside tables (0 otherwise); the inside share is
 * the window minus its outside pass. */
adx_status adx_last_kernel_split_ms(const adx_ctx *ctx, double *inside_ms, double *outside_ms);
/* Names of the fold kernel(s) and of the outside pass ("" without pair terms)
 * the last adx_run_steps launched, from the engine's own dispatch choice. */
adx_status adx_last_kernel_names(const adx_ctx *ctx, char *inside, int inside_len, char *outside, int outside_len);

adx_status adx_walkers_download(adx_ctx *ctx, char *seqs, double *scores, int64_t *counters);

/* Fold and score every walker's CURRENT configuration from scratch with the
 * MC step's own kernels (the same inside, outside and combine launches as
 * adx_run_steps, no stored tables read), adopt the fresh tables and write the
 * fresh scores[W] (and term_values[W*n_terms*max(1,n_contexts)], optional).
 * The stored scores are left alone: a caller compares the two to check that
 * incremental refolds equal scratch folds bit for bit.  adx_walkers_init
 * computes the walkers' first scores this way (sampling.cc:40).
 * State the call overwrites: each walker's table slot pointer (cur_slot flips
 * to the fresh tables) and valid byte (set), the proposal buffers of the last
 * step (proposed sequences and scores, changed flags, the launch-order list)
 * and, with base-pair terms, the pair-probability and per-variant energy
 * scratch -- so read a step's proposals before rescoring. */
adx_status adx_walkers_rescore(adx_ctx *ctx, double *scores, double *term_values);

/* Replica exchange (BASELINE config 5): copy the walkers' configurations --
 * sequence codes (W*N bytes, 1..4 = A,C,G,U) and scores (W doubles) -- to or
 * from caller-owned DEVICE buffers on the context's GPU (e.g. torch tensors
 * swapped between ranks over RCCL).  RNG streams, counters and thermostat
 * state stay with the walker slot: a swap moves configurations between
 * temperatures.  An imported walker folds from scratch until one of its
 * proposals is accepted; from then on it refolds incrementally on that
 * proposal's tables.
 *
 * adx_walkers_export / adx_walkers_import are synchronous: export returns with
 * the buffers written; the caller's own writes to the buffers must be complete
 * (its stream synchronized) before adx_walkers_import. */
adx_status adx_walkers_export(adx_ctx *ctx, void *dev_seqs, void *dev_scores);
adx_status adx_walkers_import(adx_ctx *ctx, const void *dev_seqs, const void *dev_scores);
/* Stream-ordered forms, no host synchronisation: `stream` / `producer_stream`
 * is the caller's HIP stream that reads / writes the buffers (e.g. torch's
 * current stream; NULL is the null stream -- a valid stream, not "none").
 * The copies run on the context's stream after the work already queued on the
 * caller's stream, and the caller's stream waits for the copies before its
 * later work (so it may read the exported buffers, and overwrite the imported
 * ones, right away).  Use the synchronous pair above for "no stream". */
adx_status adx_walkers_export_on(adx_ctx *ctx, void *dev_seqs, void *dev_scores, void *stream);
adx_status adx_walkers_import_after(adx_ctx *ctx, const void *dev_seqs, const void *dev_scores,
                                    void *producer_stream);
/* Temperature of an ADX_THERMO_FIXED context (one rung of a replica ladder). */
adx_status adx_set_temperature(adx_ctx *ctx, double t);

/* Parity entry point: score W sequences (W*N chars) without moving.
 * scores[W]; term_values[W*n_terms*max(1,n_contexts)] (optional);
 * dG[W*n_variants] ensemble energies (kcal/mol, float, optional). */
adx_status adx_score_batch(adx_ctx *ctx, int n_walkers, const char *seqs, double *scores,
                           double *term_values, float *dG);

/* Base-pair probability matrices of W sequences (W*N chars) for one
 * (context, condition) unconstrained fold: probs = W * L * L doubles, L the
 * folded (context-padded) length, row-major, symmetric, zero diagonal --
 * probs[w*L*L + (i-1)*L + (j-1)] = fc->exp_matrices->probs[iindx[i]-j]
 * (scoring.cc:47-50).  context = 0 without contexts. */
adx_status adx_bppm_batch(adx_ctx *ctx, int n_walkers, const char *seqs, int condition, int context,
                          double *probs);

/* Variant v of the score: which (context, condition, macrostate or -1). */
adx_status adx_variant_desc(const adx_ctx *ctx, int v, int *context, int *condition,
                            int *macrostate);

#ifdef __cplusplus
}
#endif
#endif
