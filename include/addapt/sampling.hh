// addapt-amd C++ host API: Monte Carlo sampling (reference include/sampling.hh).
//
// MonteCarlo::apply(device, rng) is the reference's single-walker loop
// (sampling.cc:22-107) with folds on the GPU (GpuRnaFold).  When the score
// function, move set and thermostat are the built-in ones (everything the
// config files can express), MonteCarlo::apply(device, seed) and
// MonteCarlo::apply_batch run the fused GPU engine instead (adx_ctx_* /
// adx_run_steps): the same trajectory per walker, thousands of walkers at once.
#pragma once

#include <cstdint>
#include <fstream>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "addapt/model.hh"
#include "addapt/scoring.hh"

namespace addapt {

class MonteCarlo;
using MonteCarloPtr = std::shared_ptr<MonteCarlo>;
class Move;
using MovePtr = std::shared_ptr<Move>;
using MoveList = std::vector<MovePtr>;
class Thermostat;
using ThermostatPtr = std::shared_ptr<Thermostat>;
class Reporter;
using ReporterPtr = std::shared_ptr<Reporter>;
using ReporterList = std::vector<ReporterPtr>;

enum class OutcomeEnum { REJECT, ACCEPT_WORSENED, ACCEPT_UNCHANGED, ACCEPT_IMPROVED };

struct MonteCarloStep {
    int i = -1, num_steps = 0;
    DevicePtr current_device, proposed_device;
    MovePtr move;
    EvaluatedScoreFunction score_table;
    double current_score = 0, proposed_score = 0, score_diff = 0;
    double temperature = 0, metropolis_criterion = 0, random_threshold = 0;
    OutcomeEnum outcome = OutcomeEnum::ACCEPT_UNCHANGED;
    std::map<OutcomeEnum, int> outcome_counters;
};

const std::map<char, char> COMPLEMENTARY_NUCS = {{'A', 'U'}, {'G', 'C'}, {'C', 'G'}, {'U', 'A'}};

bool can_be_mutated(DeviceConstPtr device, int i);
bool can_be_freely_mutated(DeviceConstPtr device, int i);
/// set position i to base and every macrostate partner to its complement,
/// recursively (sampling.cc:195-282); throws std::string on conflicts
void mutate_recursively(DevicePtr device, int i, char base);

class Move {
public:
    virtual ~Move() = default;
    virtual string name() const = 0;
    virtual void apply(DevicePtr device, std::mt19937 &rng) const = 0;
};

/// pick a freely mutable position uniformly, then a base from "ACGU"
class UnbiasedMutationMove : public Move {
public:
    string name() const override { return "UnbiasedMutation"; }
    void apply(DevicePtr device, std::mt19937 &rng) const override;
};

class Thermostat {
public:
    virtual ~Thermostat() = default;
    virtual double adjust(MonteCarloStep const &step) = 0;
};

class FixedThermostat : public Thermostat {
public:
    explicit FixedThermostat(double t) : t_(t) {}
    double adjust(MonteCarloStep const &) override { return t_; }
    double temperature() const { return t_; }
    void temperature(double t) { t_ = t; }

private:
    double t_;
};

/// T(i) = ((lo - hi) / N) * (i mod N) + hi  (sampling.cc:332-338)
class AnnealingThermostat : public Thermostat {
public:
    AnnealingThermostat(int cycle_len, double hi, double lo) : n_(cycle_len), hi_(hi), lo_(lo) {}
    double adjust(MonteCarloStep const &step) override;
    int cycle_len() const { return n_; }
    double max_temperature() const { return hi_; }
    double min_temperature() const { return lo_; }

private:
    int n_;
    double hi_, lo_;
};

/// every `period` scored steps T = max(median(score_diff) / ln(rate), 0)
/// (sampling.cc:381-401)
class AutoScalingThermostat : public Thermostat {
public:
    AutoScalingThermostat(double rate = 0.5, unsigned period = 100, double t0 = 1.0)
        : t_(t0), rate_(rate), period_(period) {}
    double adjust(MonteCarloStep const &step) override;
    double target_acceptance_rate() const { return rate_; }
    unsigned training_period() const { return period_; }
    double initial_temperature() const { return t0_; }

private:
    double t_, rate_;
    unsigned period_;
    double t0_ = t_;
    std::vector<double> train_;
};

class Reporter {
public:
    virtual ~Reporter() = default;
    virtual void start(MonteCarloStep const &) {}
    virtual void update(MonteCarloStep const &) {}
    virtual void finish(MonteCarloStep const &) {}
};

class ProgressReporter : public Reporter {
public:
    void update(MonteCarloStep const &step) override;
};

/// The reference's trajectory format (sampling.cc:427-494), one row per
/// `interval` steps.
class TsvTrajectoryReporter : public Reporter {
public:
    TsvTrajectoryReporter(string path, int interval) : path_(path), interval_(interval) {}
    void start(MonteCarloStep const &step) override;
    void update(MonteCarloStep const &step) override;
    void finish(MonteCarloStep const &step) override;

private:
    string path_;
    int interval_;
    std::ofstream tsv_;
};

/// one walker's result of a batched run
struct WalkerResult {
    DevicePtr device;
    double score;
    std::map<OutcomeEnum, long long> outcome_counters;
};

class MonteCarlo {
public:
    MonteCarlo();
    /// the reference loop; every score evaluation folds on the GPU
    DevicePtr apply(DevicePtr device, std::mt19937 &rng) const;
    /// mt19937(seed): the fused GPU engine when the setup is built-in, else
    /// the reference loop
    DevicePtr apply(DevicePtr device, uint32_t seed) const;
    /// W independent walkers (seeds[w]) on one GPU; reporters are not called
    std::vector<WalkerResult> apply_batch(DevicePtr device, const std::vector<uint32_t> &seeds,
                                          int gpu = 0) const;
    /// true if the fused GPU engine can run this setup
    bool gpu_expressible() const;

    int num_steps() const { return steps_; }
    void num_steps(int n) { steps_ = n; }
    ThermostatPtr thermostat() const { return thermostat_; }
    void thermostat(ThermostatPtr t) { thermostat_ = t; }
    ScoreFunctionPtr scorefxn() const { return scorefxn_; }
    void scorefxn(ScoreFunctionPtr s) { scorefxn_ = s; }
    MoveList moves() const { return moves_; }
    void add_move(MovePtr m) { moves_.push_back(m); }
    void operator+=(MovePtr m) { add_move(m); }
    ReporterList reporters() const { return reporters_; }
    void add_reporter(ReporterPtr r) { reporters_.push_back(r); }
    void operator+=(ReporterPtr r) { add_reporter(r); }
    void gpu(int g) { gpu_ = g; }

private:
    int steps_;
    ThermostatPtr thermostat_;
    ScoreFunctionPtr scorefxn_;
    MoveList moves_;
    ReporterList reporters_;
    int gpu_ = 0;
};

}  // namespace addapt

namespace std {
ostream &operator<<(ostream &, const addapt::OutcomeEnum &);
}
