/* CPU restatement of addapt's Monte Carlo layer (TEST INFRASTRUCTURE ONLY):
 * RNG streams, UnbiasedMutationMove, mutate_recursively, thermostats,
 * ScoreFunction / MacrostateProbTerm and MonteCarlo::apply.
 * Reference: /root/reference/src/sampling.cc, src/scoring.cc, src/model.cc. */
#include <ctype.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "adx_oracle.h"

/* ------------------------------------------------------------------ RNG */
/* std::mt19937 (seed_seq-free constructor). */
void orc_mt_seed(orc_mt *g, uint32_t seed) {
    g->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
    g->idx = 624;
}

static void mt_twist(orc_mt *g) {
    for (int i = 0; i < 624; i++) {
        uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
        g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
}

uint32_t orc_mt_next(orc_mt *g) {
    if (g->idx >= 624) mt_twist(g);
    uint32_t y = g->mt[g->idx++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* libstdc++-11 uniform_int_distribution<int>::operator() for a 32-bit URBG:
 * range < 2^32 -> Lemire nearly-divisionless (bits/uniform_int_dist.h). */
int orc_uniform_int(orc_mt *g, int a, int b) {
    uint32_t urange = (uint32_t)b - (uint32_t)a;
    if (urange == 0xffffffffu) return (int)((uint32_t)a + orc_mt_next(g));
    uint32_t uerange = urange + 1u;
    uint64_t product = (uint64_t)orc_mt_next(g) * (uint64_t)uerange;
    uint32_t low = (uint32_t)product;
    if (low < uerange) {
        uint32_t threshold = (uint32_t)(-uerange) % uerange;
        while (low < threshold) {
            product = (uint64_t)orc_mt_next(g) * (uint64_t)uerange;
            low = (uint32_t)product;
        }
    }
    return (int)((uint32_t)a + (uint32_t)(product >> 32));
}

/* generate_canonical<double, 53>(mt19937): two draws, (o1 + o2*2^32) / 2^64 */
double orc_canonical(orc_mt *g) {
    double r = 4294967296.0;
    double sum = (double)orc_mt_next(g);
    sum += (double)orc_mt_next(g) * r;
    double ret = sum / (r * r);
    if (ret >= 1.0) ret = nextafter(1.0, 0.0);
    return ret;
}

/* ----------------------------------------------------------- the move */
int orc_can_be_mutated(const char *seq, int pos) { return isupper((unsigned char)seq[pos]) != 0; }

int orc_can_be_freely_mutated(const char *seq, int n, const char *const *ms, int nm, int pos) {
    (void)n;
    if (!orc_can_be_mutated(seq, pos)) return 0;
    for (int m = 0; m < nm; m++)
        if (ms[m][pos] == ')') return 0;
    return 1;
}

static char complement(char b) {
    switch (b) {
    case 'A': return 'U';
    case 'U': return 'A';
    case 'G': return 'C';
    case 'C': return 'G';
    default: return 0;
    }
}

static int mutate_rec(char *seq, int n, const char *const *ms, int nm, int pos, char base,
                      unsigned char *done) {
    seq[pos] = base;
    done[pos] = 1;
    for (int m = 0; m < nm; m++) {
        const char *mac = ms[m];
        char open, close;
        int step;
        if (mac[pos] == '(') { open = '('; close = ')'; step = 1; }
        else if (mac[pos] == ')') { open = ')'; close = '('; step = -1; }
        else continue;
        int level = 1, partner = pos;
        while (level != 0) {
            partner += step;
            if (partner < 0 || partner >= n) return ORC_MUT_MISMATCHED_BRACKET;
            level += (mac[partner] == open);
            level -= (mac[partner] == close);
        }
        if (!orc_can_be_mutated(seq, partner)) return ORC_MUT_IMMUTABLE_PARTNER;
        char comp = complement(base);
        if (!comp) return ORC_MUT_UNSATISFIABLE; /* COMPLEMENTARY_NUCS.at() throws */
        if (!done[partner]) {
            int rc = mutate_rec(seq, n, ms, nm, partner, comp, done);
            if (rc) return rc;
        } else if (seq[partner] != comp) {
            return ORC_MUT_UNSATISFIABLE;
        }
    }
    return ORC_MUT_OK;
}

int orc_mutate_recursively(char *seq, int n, const char *const *ms, int nm, int pos, char base) {
    unsigned char *done = (unsigned char *)calloc(n ? n : 1, 1);
    int rc = mutate_rec(seq, n, ms, nm, pos, base, done);
    free(done);
    return rc;
}

/* ------------------------------------------------------ score function */
/* ViennaRnaFold::macrostate_prob (scoring.cc:53-71): both energies come back
 * from vrna_pf as float. */
static double macrostate_prob(const orc_params *P, const char *seq, const char *cst,
                              const orc_motif *motif) {
    float g_tot = (float)orc_pf_energy(P, seq, NULL, motif);
    float g_act = (float)orc_pf_energy(P, seq, cst, motif);
    double kT = orc_kT_cal() / 1000.0;
    return exp(((double)g_tot - (double)g_act) / kT);
}

static double evaluate_terms(const orc_scorefxn *sf, const char *seq, const char *const *ms,
                             int off, double *tv) {
    double score = 0.0;
    const int L = (int)strlen(seq);
    double *bpp[2] = {NULL, NULL};   /* per condition, computed on first use (scoring.cc:41-44) */
    for (int t = 0; t < sf->n_terms; t++) {
        const orc_term *T = &sf->terms[t];
        const orc_motif *motif = (T->condition == 1) ? sf->aptamer : NULL;
        double p;
        if (T->kind == 1) {
            /* ViennaRnaFold::base_pair_prob (scoring.cc:37-51): unconstrained ensemble */
            double **B = &bpp[T->condition == 1];
            if (!*B) {
                *B = (double *)malloc(sizeof(double) * (size_t)L * L);
                orc_bppm(sf->P, seq, NULL, motif, *B);
            }
            int a = T->pair_i + off, b = T->pair_j + off;
            p = (a != b && a >= 0 && b >= 0 && a < L && b < L) ? (*B)[(size_t)a * L + b] : 0.0;
        } else if (sf->mode == 1) {
            /* MFE image of macrostate_prob: float-rounded like vrna_mfe's return */
            double gt = (float)orc_mfe_energy(sf->P, seq, NULL, motif);
            double ga = (float)orc_mfe_energy(sf->P, seq, ms[T->macrostate], motif);
            p = exp((gt - ga) / (orc_kT_cal() / 1000.0));
        } else {
            p = macrostate_prob(sf->P, seq, ms[T->macrostate], motif);
        }
        if (!T->favorable) p = 1.0 - p;
        double v = log(p);
        if (tv) tv[t] = v;
        score += T->weight * v;
    }
    free(bpp[0]);
    free(bpp[1]);
    return score;
}

double orc_score(const orc_scorefxn *sf, const char *seq, int n, const char *const *ms, int nm,
                 double *tv) {
    if (sf->n_contexts == 0) {
        char *s = (char *)malloc(n + 1);
        memcpy(s, seq, n);
        s[n] = 0;
        double r = evaluate_terms(sf, s, ms, 0, tv);
        free(s);
        return r;
    }
    double score = 0.0;
    for (int c = 0; c < sf->n_contexts; c++) {
        const char *b = sf->contexts[c].before, *a = sf->contexts[c].after;
        int lb = (int)strlen(b), la = (int)strlen(a), L = lb + n + la;
        char *s = (char *)malloc(L + 1);
        memcpy(s, b, lb);
        memcpy(s + lb, seq, n);
        memcpy(s + lb + n, a, la);
        s[L] = 0;
        char **pm = (char **)malloc(sizeof(char *) * (nm ? nm : 1));
        for (int m = 0; m < nm; m++) {
            pm[m] = (char *)malloc(L + 1);
            memset(pm[m], '.', L);
            memcpy(pm[m] + lb, ms[m], n);
            pm[m][L] = 0;
        }
        score += evaluate_terms(sf, s, (const char *const *)pm, lb, tv ? tv + c * sf->n_terms : NULL);
        for (int m = 0; m < nm; m++) free(pm[m]);
        free(pm);
        free(s);
    }
    return score;
}

/* ------------------------------------------------------ Monte Carlo */
/* std::nth_element(first, first + k, first + n) over doubles with operator<,
 * restated from libstdc++ 11 (the toolchain SURVEY §8 A11 pins):
 * <bits/stl_algo.h> __introselect / __unguarded_partition_pivot /
 * __move_median_to_first / __insertion_sort and <bits/stl_heap.h>
 * __heap_select / __make_heap / __adjust_heap / __push_heap.  The order of
 * comparisons and swaps is kept step for step, so the element that lands at
 * position k is the one libstdc++ selects even among equal keys (+0.0 vs -0.0)
 * and with NaNs (which make '<' no strict weak order).  The reference calls
 * it from AutoScalingThermostat::adjust (sampling.cc:389-393). */
static void nth_swap(double *a, long i, long j) { double t = a[i]; a[i] = a[j]; a[j] = t; }

static void nth_push_heap(double *a, long hole, long top, double v) {
    long parent = (hole - 1) / 2;
    while (hole > top && a[parent] < v) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = v;
}

static void nth_adjust_heap(double *a, long hole, long len, double v) {
    const long top = hole;
    long child = hole;
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
    nth_push_heap(a, hole, top, v);
}

static void nth_heap_select(double *a, long mid, long last) {
    if (mid >= 2)
        for (long parent = (mid - 2) / 2;; parent--) {
            nth_adjust_heap(a, parent, mid, a[parent]);
            if (parent == 0) break;
        }
    for (long i = mid; i < last; i++)
        if (a[i] < a[0]) {
            double v = a[i];
            a[i] = a[0];
            nth_adjust_heap(a, 0, mid, v);
        }
}

static void nth_insertion_sort(double *a, long first, long last) {
    if (first == last) return;
    for (long i = first + 1; i != last; i++) {
        double v = a[i];
        if (v < a[first]) {
            memmove(a + first + 1, a + first, sizeof(double) * (size_t)(i - first));
            a[first] = v;
        } else {
            long hole = i, prev = i - 1;
            while (v < a[prev]) {
                a[hole] = a[prev];
                hole = prev;
                prev--;
            }
            a[hole] = v;
        }
    }
}

static void nth_median_to_first(double *x, long r, long a, long b, long c) {
    if (x[a] < x[b]) {
        if (x[b] < x[c]) nth_swap(x, r, b);
        else if (x[a] < x[c]) nth_swap(x, r, c);
        else nth_swap(x, r, a);
    } else if (x[a] < x[c]) nth_swap(x, r, a);
    else if (x[b] < x[c]) nth_swap(x, r, c);
    else nth_swap(x, r, b);
}

static long nth_partition_pivot(double *a, long first, long last) {
    long mid = first + (last - first) / 2;
    nth_median_to_first(a, first, first + 1, mid, last - 1);
    long lo = first + 1, hi = last;
    const long pivot = first;
    for (;;) {
        while (a[lo] < a[pivot]) lo++;
        hi--;
        while (a[pivot] < a[hi]) hi--;
        if (!(lo < hi)) return lo;
        nth_swap(a, lo, hi);
        lo++;
    }
}

void orc_nth_element(double *a, long k, long n) {
    if (n == 0 || k == n) return;
    long first = 0, last = n;
    int lg = 63 - __builtin_clzll((unsigned long long)n);
    long depth = 2L * lg;
    while (last - first > 3) {
        if (depth == 0) {
            nth_heap_select(a + first, k + 1 - first, last - first);
            nth_swap(a, first, k);
            return;
        }
        --depth;
        long cut = nth_partition_pivot(a, first, last);
        if (cut <= k) first = cut;
        else last = cut;
    }
    nth_insertion_sort(a, first, last);
}

/* std::max(t, 0.0) = (t < 0.0) ? 0.0 : t  (<bits/stl_algobase.h>): keeps -0.0
 * and NaN, as AutoScalingThermostat::adjust does (sampling.cc:395-396). */
double orc_auto_clamp(double t) { return (t < 0.0) ? 0.0 : t; }

int orc_mc_run(const orc_scorefxn *sf, char *seq, int n, const char *const *ms, int nm,
               const orc_thermostat *th, uint32_t seed, int num_steps, double *final_score,
               int64_t *counters, orc_trace *trace, const orc_mc_opts *opts) {
    /* MonteCarlo::apply (sampling.cc:22-107).  rng (stream A) and the copy
     * bound into `random` (stream C) both start from mt19937(seed); the
     * randmove copy (stream B) always yields 0 with one move and is skipped. */
    orc_mt A, C;
    orc_mt_seed(&A, seed);
    orc_mt_seed(&C, seed);
    char *cur = (char *)malloc(n + 1), *prop = (char *)malloc(n + 1);
    memcpy(cur, seq, n);
    cur[n] = 0;
    prop[n] = 0;
    int *mut = (int *)malloc(sizeof(int) * (n ? n : 1)), M = 0;
    for (int i = 0; i < n; i++)
        if (orc_can_be_freely_mutated(cur, n, ms, nm, i)) mut[M++] = i;
    double current = orc_score(sf, cur, n, ms, nm, NULL);
    double score_diff = 0.0; /* uninitialised in the reference (sampling.hh:95-104) */
    double temperature = th->t_fixed;
    double *training = (double *)malloc(sizeof(double) * (th->period > 0 ? th->period + 1 : 1));
    int ntrain = 0;
    double auto_T = th->t_init;
    int64_t cnt[4] = {0, 0, 0, 0};
    int rc = ORC_MUT_OK;
    for (int i = 0; i < num_steps; i++) {
        /* Thermostat::adjust (sampling.cc:309-401) */
        if (th->kind == 0) temperature = th->t_fixed;
        else if (th->kind == 1) {
            int N = th->cycle_len;
            temperature = ((th->t_lo - th->t_hi) / N) * (i % N) + th->t_hi;
        } else {
            training[ntrain++] = score_diff;
            if ((unsigned)ntrain >= (unsigned)th->period) {
                int k = ntrain / 2;
                orc_nth_element(training, k, ntrain);
                auto_T = orc_auto_clamp(training[k] / log(th->target_rate));
                ntrain = 0;
            }
            temperature = auto_T;
        }
        memcpy(prop, cur, n);
        if (M == 0) { rc = ORC_MUT_UNSATISFIABLE; break; } /* vector index out of range */
        int pick = orc_uniform_int(&A, 0, M - 1);
        int pos = mut[pick];
        char base = "ACGU"[orc_uniform_int(&A, 0, 3)];
        rc = orc_mutate_recursively(prop, n, ms, nm, pos, base);
        if (rc) break;
        int outcome;
        double prop_score = NAN, u = NAN;
        if (memcmp(prop, cur, n) == 0) {
            outcome = ORC_ACCEPT_UNCHANGED;
        } else {
            prop_score = orc_score(sf, prop, n, ms, nm, NULL);
            score_diff = prop_score - current;
            double crit = exp(score_diff / temperature);
            u = orc_canonical(&C);
            int reject = crit < u;
            if (opts && opts->forced_outcome && fabs(crit - u) <= opts->tie_eps)
                reject = opts->forced_outcome[i] == ORC_REJECT;
            if (reject) outcome = ORC_REJECT;
            else {
                outcome = score_diff > 0 ? ORC_ACCEPT_IMPROVED : ORC_ACCEPT_WORSENED;
                memcpy(cur, prop, n);
                current = prop_score;
            }
        }
        cnt[outcome]++;
        if (trace) {
            if (trace->pos) trace->pos[i] = pos;
            if (trace->base) trace->base[i] = base;
            if (trace->outcome) trace->outcome[i] = outcome;
            if (trace->temperature) trace->temperature[i] = temperature;
            if (trace->proposed_score) trace->proposed_score[i] = prop_score;
            if (trace->current_score) trace->current_score[i] = current;
            if (trace->random_threshold) trace->random_threshold[i] = u;
            if (trace->seqs) memcpy(trace->seqs + (size_t)i * n, cur, n);
        }
    }
    memcpy(seq, cur, n);
    if (final_score) *final_score = current;
    if (counters)
        for (int k = 0; k < 4; k++) counters[k] = cnt[k];
    free(cur); free(prop); free(mut); free(training);
    return rc;
}

double orc_mc_run_batch(const orc_scorefxn *sf, char *seqs, int n, int W, const char *const *ms,
                        int nm, const orc_thermostat *th, const uint32_t *seeds, int num_steps,
                        int n_threads, int64_t *counters_total) {
    struct timespec t0, t1;
    int64_t tot[4] = {0, 0, 0, 0};
    clock_gettime(CLOCK_MONOTONIC, &t0);
#ifdef _OPENMP
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 1)
#endif
    for (int w = 0; w < W; w++) {
        int64_t c[4];
        double fs;
        orc_mc_run(sf, seqs + (size_t)w * n, n, ms, nm, th, seeds[w], num_steps, &fs, c, NULL, NULL);
#ifdef _OPENMP
#pragma omp critical
#endif
        for (int k = 0; k < 4; k++) tot[k] += c[k];
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (counters_total)
        for (int k = 0; k < 4; k++) counters_total[k] = tot[k];
    (void)n_threads;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
