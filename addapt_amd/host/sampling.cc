// Monte Carlo sampling (reference src/sampling.cc semantics): the
// single-walker reference loop, and the batched path over the fused GPU
// engine (adx_ctx_* / adx_run_steps) for built-in setups.
#include "addapt/sampling.hh"

#include <algorithm>
#include <cctype>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>
#include <limits>
#include <unistd.h>

#include "gpu.hh"

namespace addapt {

static string fmt(const char *f, ...) __attribute__((format(printf, 1, 2)));
static string fmt(const char *f, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, f);
    std::vsnprintf(buf, sizeof buf, f, ap);
    va_end(ap);
    return buf;
}

// ---------------------------------------------------------------- moves
bool can_be_mutated(DeviceConstPtr device, int i) { return std::isupper(static_cast<unsigned char>(device->seq()[i])) != 0; }

bool can_be_freely_mutated(DeviceConstPtr device, int i) {
    if (!can_be_mutated(device, i)) return false;
    for (auto &m : device->macrostates())
        if (m.second[i] == ')') return false;   // mutated as a unit with its '(' partner
    return true;
}

static void mutate_rec(DevicePtr device, int pos, char base, std::vector<bool> &done) {
    device->mutate(pos, base);
    done[pos] = true;
    for (auto &m : device->macrostates()) {
        const string &ms = m.second;
        int step;
        char open, close;
        if (ms[pos] == '(') { open = '('; close = ')'; step = 1; }
        else if (ms[pos] == ')') { open = ')'; close = '('; step = -1; }
        else continue;
        int level = 1, partner = pos;
        while (level != 0) {
            partner += step;
            if (partner < 0 || partner >= static_cast<int>(ms.size()))
                throw fmt("mismatched base-pair in '%s' macrostate: '%s'", m.first.c_str(), ms.c_str());
            level += ms[partner] == open;
            level -= ms[partner] == close;
        }
        if (!can_be_mutated(device, partner))
            throw fmt("position '%d' can be mutated, but it's base-paired to position '%d' which can't be.", pos, partner);
        const char comp = COMPLEMENTARY_NUCS.at(base);
        if (!done[partner]) mutate_rec(device, partner, comp, done);
        else if (device->seq()[partner] != comp) throw string("no way to satisfy all base pairing constraints.");
    }
}

void mutate_recursively(DevicePtr device, int i, char base) {
    std::vector<bool> done(device->len(), false);
    mutate_rec(device, i, base, done);
}

void UnbiasedMutationMove::apply(DevicePtr device, std::mt19937 &rng) const {
    std::vector<int> free_pos;
    for (int i = 0; i < device->len(); i++)
        if (can_be_freely_mutated(device, i)) free_pos.push_back(i);
    if (free_pos.empty()) throw string("no freely mutable positions");
    const int pick = free_pos[std::uniform_int_distribution<>(0, int(free_pos.size()) - 1)(rng)];
    const char base = "ACGU"[std::uniform_int_distribution<>(0, 3)(rng)];
    mutate_recursively(device, pick, base);
}

// ---------------------------------------------------------------- thermostats
double AnnealingThermostat::adjust(MonteCarloStep const &step) {
    return ((lo_ - hi_) / n_) * (step.i % n_) + hi_;
}

double AutoScalingThermostat::adjust(MonteCarloStep const &step) {
    train_.push_back(step.score_diff);
    if (train_.size() >= period_) {
        const size_t n = train_.size() / 2;
        std::nth_element(train_.begin(), train_.begin() + n, train_.end());
        t_ = std::max(train_[n] / std::log(rate_), 0.0);
        train_.clear();
    }
    return t_;
}

// ---------------------------------------------------------------- reporters
void ProgressReporter::update(MonteCarloStep const &step) {
    if (!isatty(fileno(stdout))) return;
    std::cout << "\033[2K\r[" << step.i + 1 << "/" << step.num_steps << "]";
    if (step.i + 1 == step.num_steps) std::cout << std::endl;
    else std::cout << std::flush;
}

void TsvTrajectoryReporter::start(MonteCarloStep const &step) {
    tsv_.open(path_);
    if (!tsv_.is_open()) throw fmt("couldn't open '%s' for writing", path_.c_str());
    tsv_ << "#\tinitial_seq\t" << step.current_device->seq() << "\n";
    tsv_ << "step\tnum_steps\tcurrent_score\tproposed_score\t";
    for (auto &row : step.score_table) tsv_ << "term_weight[" << row.name << "]\tterm_value[" << row.name << "]\t";
    tsv_ << "score_diff\ttemperature\tmetropolis_criterion\trandom_threshold\tmove\toutcome\tcurrent_seq\tproposed_seq\t"
         << std::endl;
}

void TsvTrajectoryReporter::update(MonteCarloStep const &step) {
    if (step.i % interval_ != 0) return;
    tsv_ << step.i << "\t" << step.num_steps << "\t" << step.current_score << "\t" << step.proposed_score << "\t";
    for (auto &row : step.score_table) tsv_ << row.weight << "\t" << row.term << "\t";
    tsv_ << step.score_diff << "\t" << step.temperature << "\t" << step.metropolis_criterion << "\t"
         << step.random_threshold << "\t" << step.move->name() << "\t" << step.outcome << "\t"
         << step.current_device->seq() << "\t" << step.proposed_device->seq() << "\t" << std::endl;
}

void TsvTrajectoryReporter::finish(MonteCarloStep const &) { tsv_.close(); }

// ---------------------------------------------------------------- reference loop
MonteCarlo::MonteCarlo()
    : steps_(0), thermostat_(std::make_shared<FixedThermostat>(1)), scorefxn_(std::make_shared<ScoreFunction>()) {}

// sampling.cc:22-107.  The move draws from `rng` itself; the move picker and
// the Metropolis uniform draw from copies of its state at entry (std::bind
// copies the engine), exactly as the reference.
DevicePtr MonteCarlo::apply(DevicePtr device, std::mt19937 &rng) const {
    if (moves_.empty()) return device;
    MonteCarloStep step;
    step.num_steps = steps_;
    step.i = -1;
    step.current_device = device;
    auto random = std::bind(std::uniform_real_distribution<>(), rng);
    auto randmove = std::bind(std::uniform_int_distribution<>(0, int(moves_.size()) - 1), rng);
    step.current_score = scorefxn_->evaluate(step.current_device, step.score_table);
    step.proposed_score = step.current_score;
    for (auto o : {OutcomeEnum::REJECT, OutcomeEnum::ACCEPT_WORSENED, OutcomeEnum::ACCEPT_UNCHANGED,
                   OutcomeEnum::ACCEPT_IMPROVED})
        step.outcome_counters[o] = 0;
    for (auto &r : reporters_) r->start(step);
    for (step.i = 0; step.i < step.num_steps; step.i++) {
        step.temperature = thermostat_->adjust(step);
        step.proposed_device = step.current_device->copy();
        step.move = moves_[randmove()];
        step.move->apply(step.proposed_device, rng);
        if (step.current_device->seq() == step.proposed_device->seq()) {
            step.outcome = OutcomeEnum::ACCEPT_UNCHANGED;
        } else {
            step.proposed_score = scorefxn_->evaluate(step.proposed_device, step.score_table);
            step.score_diff = step.proposed_score - step.current_score;
            step.metropolis_criterion = std::exp(step.score_diff / step.temperature);
            step.random_threshold = random();
            if (step.metropolis_criterion < step.random_threshold) {
                step.outcome = OutcomeEnum::REJECT;
            } else {
                step.outcome = step.score_diff > 0 ? OutcomeEnum::ACCEPT_IMPROVED : OutcomeEnum::ACCEPT_WORSENED;
                step.current_device = step.proposed_device;
                step.current_score = step.proposed_score;
            }
        }
        step.outcome_counters[step.outcome] += 1;
        for (auto &r : reporters_) r->update(step);
    }
    for (auto &r : reporters_) r->finish(step);
    return step.current_device;
}

// ---------------------------------------------------------------- GPU engine path
bool MonteCarlo::gpu_expressible() const {
    if (moves_.size() != 1 || !std::dynamic_pointer_cast<UnbiasedMutationMove>(moves_[0])) return false;
    if (!std::dynamic_pointer_cast<FixedThermostat>(thermostat_) &&
        !std::dynamic_pointer_cast<AnnealingThermostat>(thermostat_) &&
        !std::dynamic_pointer_cast<AutoScalingThermostat>(thermostat_))
        return false;
    if (scorefxn_->terms().empty()) return false;
    for (auto &t : scorefxn_->terms())
        if (!std::dynamic_pointer_cast<MacrostateProbTerm>(t)) return false;
    return true;
}

namespace {
struct EngineSetup {
    std::vector<string> names, macro;
    std::vector<const char *> macro_c;
    std::vector<adx_term> terms;
    std::vector<string> ctx_b, ctx_a;
    std::vector<adx_context_desc> ctx;
    string seq, apt_seq, apt_fold;
    adx_run_desc d{};
};

void build_setup(const MonteCarlo &mc, DeviceConstPtr device, int g, EngineSetup &e) {
    if (device->context() && (!device->context()->before().empty() || !device->context()->after().empty()))
        throw string("the engine folds devices without a context (contexts belong to the score function)");
    e.seq = device->raw_seq();
    e.names = device->macrostate_names();
    for (auto &n : e.names) e.macro.push_back(device->macrostate(n));
    for (auto &m : e.macro) e.macro_c.push_back(m.c_str());
    for (auto &t : mc.scorefxn()->terms()) {
        auto m = std::dynamic_pointer_cast<MacrostateProbTerm>(t);
        auto it = std::find(e.names.begin(), e.names.end(), m->macrostate());
        if (it == e.names.end()) throw string("no macrostate named '" + m->macrostate() + "'");
        e.terms.push_back(adx_term{m->condition() == ConditionEnum::APO ? ADX_APO : ADX_HOLO,
                                   int(it - e.names.begin()), m->favorable() == FavorableEnum::YES ? 1 : 0,
                                   m->weight()});
    }
    for (auto &kv : mc.scorefxn()->contexts()) {
        e.ctx_b.push_back(kv.second->before());
        e.ctx_a.push_back(kv.second->after());
    }
    for (size_t k = 0; k < e.ctx_b.size(); k++) e.ctx.push_back(adx_context_desc{e.ctx_b[k].c_str(), e.ctx_a[k].c_str()});
    adx_run_desc &d = e.d;
    d.params = gpu::params();
    d.sequence = e.seq.c_str();
    d.n_macrostates = int(e.macro_c.size());
    d.macrostates = e.macro_c.data();
    d.n_terms = int(e.terms.size());
    d.terms = e.terms.data();
    if (auto a = mc.scorefxn()->aptamer()) {
        e.apt_seq = a->seq();
        e.apt_fold = a->fold();
        d.aptamer_seq = e.apt_seq.c_str();
        d.aptamer_fold = e.apt_fold.c_str();
        d.aptamer_energy_kcal = kT() * std::log(a->affinity() / 1e6);
    }
    d.motif_mode = ADX_MOTIF_AUTO;   // ADD in partition functions, REPLACE in MFE folds (every reference pin)
    d.n_contexts = int(e.ctx.size());
    d.contexts = e.ctx.empty() ? nullptr : e.ctx.data();
    auto th = mc.thermostat();
    if (auto f = std::dynamic_pointer_cast<FixedThermostat>(th)) {
        d.thermostat.kind = ADX_THERMO_FIXED;
        d.thermostat.t_fixed = f->temperature();
    } else if (auto a = std::dynamic_pointer_cast<AnnealingThermostat>(th)) {
        d.thermostat.kind = ADX_THERMO_ANNEAL;
        d.thermostat.cycle_len = a->cycle_len();
        d.thermostat.t_hi = a->max_temperature();
        d.thermostat.t_lo = a->min_temperature();
    } else if (auto s = std::dynamic_pointer_cast<AutoScalingThermostat>(th)) {
        d.thermostat.kind = ADX_THERMO_AUTO;
        d.thermostat.target_rate = s->target_acceptance_rate();
        d.thermostat.period = int(s->training_period());
        d.thermostat.t_init = s->initial_temperature();
    }
    d.device = g;
}
}  // namespace

std::vector<WalkerResult> MonteCarlo::apply_batch(DevicePtr device, const std::vector<uint32_t> &seeds, int g) const {
    if (!gpu_expressible()) throw string("apply_batch: the score function / moves / thermostat are not GPU-expressible");
    EngineSetup e;
    build_setup(*this, device, g, e);
    adx_ctx *raw = nullptr;
    gpu::check(adx_ctx_create(&e.d, &raw));
    gpu::CtxPtr ctx(raw);
    const int W = int(seeds.size());
    gpu::check(adx_walkers_init(ctx.get(), W, nullptr, seeds.data()));
    if (steps_ > 0) gpu::check(adx_run_steps(ctx.get(), steps_, nullptr));
    const size_t N = e.seq.size();
    std::vector<char> seqs(N * W);
    std::vector<double> scores(W);
    std::vector<int64_t> cnt(4 * size_t(W));
    gpu::check(adx_walkers_download(ctx.get(), seqs.data(), scores.data(), cnt.data()));
    std::vector<WalkerResult> out(W);
    for (int w = 0; w < W; w++) {
        out[w].device = device->copy();
        for (size_t k = 0; k < N; k++) out[w].device->mutate(int(k), seqs[size_t(w) * N + k]);
        out[w].score = scores[w];
        const OutcomeEnum o[4] = {OutcomeEnum::REJECT, OutcomeEnum::ACCEPT_WORSENED, OutcomeEnum::ACCEPT_UNCHANGED,
                                  OutcomeEnum::ACCEPT_IMPROVED};
        for (int k = 0; k < 4; k++) out[w].outcome_counters[o[k]] = cnt[size_t(w) * 4 + k];
    }
    return out;
}

// One walker on the engine, replayed through the reporters: the engine's
// per-step trace (position, base, outcome, T, proposed / current score,
// uniform draw, term values) rebuilds the reference's MonteCarloStep,
// including the values the reference leaves stale on ACCEPT_UNCHANGED steps.
DevicePtr MonteCarlo::apply(DevicePtr device, uint32_t seed) const {
    if (!gpu_expressible()) {
        std::mt19937 rng(seed);
        return apply(device, rng);
    }
    EngineSetup e;
    build_setup(*this, device, gpu_, e);
    adx_ctx *raw = nullptr;
    gpu::check(adx_ctx_create(&e.d, &raw));
    gpu::CtxPtr ctx(raw);
    gpu::check(adx_walkers_init(ctx.get(), 1, nullptr, &seed));
    MonteCarloStep step;
    step.num_steps = steps_;
    step.current_device = device;
    // initial score and table
    const int nctx = std::max<int>(1, int(e.ctx.size()));
    const int nt = int(e.terms.size()) * nctx;
    std::vector<double> tv(nt);
    double s0 = 0;
    gpu::check(adx_score_batch(ctx.get(), 1, e.seq.c_str(), &s0, tv.data(), nullptr));
    std::vector<string> names;
    std::vector<double> weights;
    if (e.ctx.empty()) {
        for (auto &t : scorefxn_->terms()) { names.push_back(t->name()); weights.push_back(t->weight()); }
    } else {
        for (auto &kv : scorefxn_->contexts())
            for (auto &t : scorefxn_->terms()) { names.push_back(kv.first + ": " + t->name()); weights.push_back(t->weight()); }
    }
    auto table = [&](const double *v) {
        EvaluatedScoreFunction t;
        for (int k = 0; k < nt; k++) t.push_back(EvaluatedScoreTerm{names[k], weights[k], v[k]});
        return t;
    };
    step.current_score = step.proposed_score = s0;
    step.score_table = table(tv.data());
    for (auto o : {OutcomeEnum::REJECT, OutcomeEnum::ACCEPT_WORSENED, OutcomeEnum::ACCEPT_UNCHANGED,
                   OutcomeEnum::ACCEPT_IMPROVED})
        step.outcome_counters[o] = 0;
    for (auto &r : reporters_) r->start(step);
    const int chunk = 4096;
    std::vector<int32_t> pos(chunk), outc(chunk);
    std::vector<char> base(chunk);
    std::vector<double> temp(chunk), prop(chunk), cur(chunk), thr(chunk), terms(size_t(chunk) * nt);
    const OutcomeEnum omap[4] = {OutcomeEnum::REJECT, OutcomeEnum::ACCEPT_WORSENED, OutcomeEnum::ACCEPT_UNCHANGED,
                                 OutcomeEnum::ACCEPT_IMPROVED};
    step.move = moves_[0];
    for (int s0i = 0; s0i < steps_; s0i += chunk) {
        const int n = std::min(chunk, steps_ - s0i);
        adx_trace tr{pos.data(), base.data(), outc.data(), temp.data(), prop.data(), cur.data(), thr.data(),
                     nt > 0 ? terms.data() : nullptr};
        gpu::check(adx_run_steps(ctx.get(), n, &tr));
        for (int k = 0; k < n; k++) {
            step.i = s0i + k;
            step.temperature = temp[k];
            step.proposed_device = step.current_device->copy();
            mutate_recursively(step.proposed_device, pos[k], base[k]);
            step.outcome = omap[outc[k]];
            if (step.outcome != OutcomeEnum::ACCEPT_UNCHANGED) {
                step.proposed_score = prop[k];
                step.score_diff = step.proposed_score - step.current_score;
                step.metropolis_criterion = std::exp(step.score_diff / step.temperature);
                step.random_threshold = thr[k];
                step.score_table = table(&terms[size_t(k) * nt]);
                if (step.outcome != OutcomeEnum::REJECT) {
                    step.current_device = step.proposed_device;
                    step.current_score = cur[k];
                }
            }
            step.outcome_counters[step.outcome] += 1;
            for (auto &r : reporters_) r->update(step);
        }
    }
    for (auto &r : reporters_) r->finish(step);
    return step.current_device;
}

}  // namespace addapt

namespace std {
ostream &operator<<(ostream &out, const addapt::OutcomeEnum &o) {
    switch (o) {
        case addapt::OutcomeEnum::REJECT: out << "REJECT"; break;
        case addapt::OutcomeEnum::ACCEPT_WORSENED: out << "ACCEPT_WORSENED"; break;
        case addapt::OutcomeEnum::ACCEPT_UNCHANGED: out << "ACCEPT_UNCHANGED"; break;
        case addapt::OutcomeEnum::ACCEPT_IMPROVED: out << "ACCEPT_IMPROVED"; break;
    }
    return out;
}
}  // namespace std
