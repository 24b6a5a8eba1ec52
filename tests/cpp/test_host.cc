// CPU tests of the C++ host mirror (no GPU call is made): the reference's
// test_model.cc, test_sampling.cc and test_scoring.cc cases restated against
// include/addapt/*.hh, plus the config reader and the TSV reporter.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "addapt/config.hh"
#include "addapt/model.hh"
#include "addapt/sampling.hh"
#include "addapt/scoring.hh"
#include "addapt/yaml.hh"

using namespace addapt;
using std::string;

static int g_fail = 0, g_pass = 0;
#define CHECK(x)                                                                          \
    do {                                                                                  \
        if (x) g_pass++;                                                                  \
        else { g_fail++; std::fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #x); } \
    } while (0)
#define CHECK_THROWS(x)                                                                   \
    do {                                                                                  \
        bool thrown_ = false;                                                             \
        try { x; } catch (...) { thrown_ = true; }                                        \
        CHECK(thrown_);                                                                   \
    } while (0)
static bool approx(double a, double b) { return std::fabs(a - b) <= 1e-9 * std::max(1.0, std::fabs(b)); }

// ------------------------------------------------------------ test_model.cc
static void test_device() {
    Device d("ACGU");
    CHECK(d.seq() == "ACGU");
    CHECK(d.len() == 4);
    CHECK(d.seq(0) == 'A' && d.seq(1) == 'C' && d.seq(2) == 'G' && d.seq(3) == 'U');
    CHECK_THROWS(d.seq(4));
    CHECK(d.seq(-1) == 'U' && d.seq(-2) == 'G' && d.seq(-3) == 'C' && d.seq(-4) == 'A');
    CHECK_THROWS(d.seq(-5));
    d.add_macrostate("a", "....");
    d.add_macrostate("b", "(())");
    CHECK(d.macrostate("a") == "....");
    CHECK(d.macrostate("b") == "(())");
    CHECK_THROWS(d.add_macrostate("c", "..."));
    DevicePtr d2 = d.copy();
    CHECK(d2->seq() == "ACGU" && d2->macrostate("a") == "...." && d2->macrostate("b") == "(())");
    Device d3("nnnn");
    d3.assign(d2);
    CHECK(d3.seq() == "ACGU" && d3.macrostate("b") == "(())");
}

static void test_device_contexts() {
    Device d("C");
    d.add_macrostate("bp", "x");
    CHECK(d.context()->before() == "" && d.context()->after() == "");
    d.context(std::make_shared<Context>("A", "GU"));
    CHECK(d.len() == 4 && d.seq() == "ACGU" && d.seq(3) == 'U');
    CHECK(d.raw_len() == 1 && d.raw_seq() == "C" && d.raw_seq(0) == 'C');
    CHECK(d.macrostate("bp") == ".x..");
    for (auto &m : d.macrostates()) CHECK(m.first == "bp" && m.second == ".x..");
    d.remove_context();
    CHECK(d.len() == 1 && d.seq() == "C" && d.macrostate("bp") == "x");
}

static void test_device_mutate() {
    Device a("AAAA");
    a.mutate(0, 'U'); CHECK(a.seq() == "UAAA");
    a.mutate(3, 'U'); CHECK(a.seq() == "UAAU");
    Device b("AAAA");
    b.mutate(-1, 'U'); CHECK(b.seq() == "AAAU");
    b.mutate(-4, 'U'); CHECK(b.seq() == "UAAU");
    CHECK_THROWS(b.mutate(4, 'U'));
    CHECK_THROWS(b.mutate(-5, 'U'));
}

static void test_aptamer() {
    Aptamer t("GAUACCAGCCGAAAGGCCCUUGGCAGC", "(...((.(((....)))....))...)", 0.320);
    CHECK(t.seq() == "GAUACCAGCCGAAAGGCCCUUGGCAGC");
    CHECK(t.fold() == "(...((.(((....)))....))...)");
    CHECK(t.affinity() == 0.320);
}

// ------------------------------------------------------------ test_sampling.cc
static void test_mutable_positions() {
    auto d = std::make_shared<Device>("UUUuuu");
    d->add_macrostate("a", "(.)(.)");
    const bool mut[] = {1, 1, 1, 0, 0, 0}, free_[] = {1, 1, 0, 0, 0, 0};
    for (int i = 0; i < 6; i++) {
        CHECK(can_be_mutated(d, i) == mut[i]);
        CHECK(can_be_freely_mutated(d, i) == free_[i]);
    }
    auto e = std::make_shared<Device>("UUUU");
    e->add_macrostate("a", "().)");
    e->add_macrostate("b", "(.))");
    const bool free2[] = {1, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        CHECK(can_be_mutated(e, i));
        CHECK(can_be_freely_mutated(e, i) == free2[i]);
    }
}

static void test_mutate_recursively() {
    struct T {
        string seq;
        std::vector<string> macro;
        string muts;
        std::vector<string> expect;
    };
    const std::vector<T> tests = {
        {"N", {"."}, "A", {"A"}},
        {"NN", {"()"}, "AG", {"AU", "CG"}},
        {"NNN", {"(.)"}, "AGU", {"ANU", "NGN", "ANU"}},
        {"NN", {"()", "()"}, "AG", {"AU", "CG"}},
        {"NNN", {"().", ".()"}, "AGU", {"AUA", "CGC", "UAU"}},
        {"NNN", {"().", "(.)"}, "AGU", {"AUU", "CGG", "AUU"}},
        {"NNNN", {"()..", "(())"}, "AGUC", {"AUAU", "CGCG", "UAUA", "GCGC"}},
        {"NNNN", {"(.).", "(())"}, "AGUC", {"AAUU", "GGCC", "AAUU", "GGCC"}},
    };
    for (auto &t : tests) {
        for (size_t i = 0; i < t.muts.size(); i++) {
            auto d = std::make_shared<Device>(t.seq);
            for (size_t x = 0; x < t.macro.size(); x++) d->add_macrostate(std::to_string(x), t.macro[x]);
            mutate_recursively(d, int(i), t.muts[i]);
            CHECK(d->seq() == t.expect[i]);
        }
    }
    auto a = std::make_shared<Device>("Nn");
    a->add_macrostate("not mutable", "()");
    CHECK_THROWS(mutate_recursively(a, 0, 'G'));
    auto b = std::make_shared<Device>("N");
    b->add_macrostate("extra open", "(");
    CHECK_THROWS(mutate_recursively(b, 0, 'G'));
    auto c = std::make_shared<Device>("N");
    c->add_macrostate("extra close", ")");
    CHECK_THROWS(mutate_recursively(c, 0, 'G'));
}

static void test_thermostats() {
    AnnealingThermostat an(300, 5.0, 0.0);
    MonteCarloStep st;
    st.i = 0; CHECK(approx(an.adjust(st), 5.0));
    st.i = 150; CHECK(approx(an.adjust(st), 2.5));
    st.i = 300; CHECK(approx(an.adjust(st), 5.0));
    st.i = 299; CHECK(approx(an.adjust(st), 5.0 - 299 * (5.0 / 300)));
    AutoScalingThermostat au(0.5, 4, 1.0);
    double diffs[] = {-1.0, -3.0, -2.0, -4.0};
    double t = 0;
    for (double x : diffs) { st.score_diff = x; t = au.adjust(st); }
    // median (nth_element at n/2 = 2) of {-1,-3,-2,-4} = -2; T = -2 / ln 0.5
    CHECK(approx(t, -2.0 / std::log(0.5)));
    auto f = thermostat_from_str("5");
    CHECK(std::dynamic_pointer_cast<FixedThermostat>(f) && approx(std::dynamic_pointer_cast<FixedThermostat>(f)->temperature(), 5));
    auto a2 = std::dynamic_pointer_cast<AnnealingThermostat>(thermostat_from_str("1 to 0 in 500 steps"));
    CHECK(a2 && a2->cycle_len() == 500 && approx(a2->max_temperature(), 1) && approx(a2->min_temperature(), 0));
    auto s2 = std::dynamic_pointer_cast<AutoScalingThermostat>(thermostat_from_str("auto 30% 50 2"));
    CHECK(s2 && approx(s2->target_acceptance_rate(), 0.3) && s2->training_period() == 50 && approx(s2->initial_temperature(), 2));
    auto s3 = std::dynamic_pointer_cast<AutoScalingThermostat>(thermostat_from_str("auto"));
    CHECK(s3 && approx(s3->target_acceptance_rate(), 0.5) && s3->training_period() == 100);
    CHECK_THROWS(thermostat_from_str("hot"));
}

// ------------------------------------------------------------ test_scoring.cc
class DummyRnaFold : public RnaFold {
public:
    explicit DummyRnaFold(double p = 0) : p_(p) {}
    double &operator[](std::pair<int, int> k) { return bp_[{std::min(k.first, k.second), std::max(k.first, k.second)}]; }
    double base_pair_prob(int a, int b) const override {
        auto it = bp_.find({std::min(a, b), std::max(a, b)});
        return it == bp_.end() ? 0.0 : it->second;
    }
    double macrostate_prob(string) const override { return p_; }

private:
    std::map<std::pair<int, int>, double> bp_;
    double p_;
};

static std::shared_ptr<RnaFold> dummy_factory(DeviceConstPtr, AptamerConstPtr) {
    return std::make_shared<DummyRnaFold>(0.5);
}

class ConstTerm : public ScoreTerm {
public:
    ConstTerm(double s, double w) : ScoreTerm("dummy", w), s_(s) {}
    double evaluate(DeviceConstPtr, RnaFold const &, RnaFold const &) const override { return s_; }

private:
    double s_;
};

class LenTerm : public ScoreTerm {
public:
    double evaluate(DeviceConstPtr d, RnaFold const &, RnaFold const &) const override { return d->len(); }
};

static void test_score_function() {
    DummyRnaFold fold;
    CHECK(fold.base_pair_prob(1, 2) == 0.0);
    fold[{1, 2}] = 0.75;
    CHECK(fold.base_pair_prob(2, 1) == 0.75);
    auto dev = std::make_shared<Device>("UUUU");
    {
        ScoreFunction sf;
        sf.fold_factory(dummy_factory);
        CHECK(approx(sf.evaluate(dev), 0));
        sf += std::make_shared<ConstTerm>(10, 1);
        CHECK(approx(sf.evaluate(dev), 10));
        sf += std::make_shared<ConstTerm>(10, 0.5);
        CHECK(approx(sf.evaluate(dev), 15));
    }
    {
        ScoreFunction sf;
        sf.fold_factory(dummy_factory);
        sf += std::make_shared<LenTerm>();
        auto u = std::make_shared<Device>("U");
        CHECK(approx(sf.evaluate(u), 1.0));
        sf.add_context("1", std::make_shared<Context>("a", ""));
        CHECK(approx(sf.evaluate(u), 2.0));
        sf.add_context("2", std::make_shared<Context>("a", "a"));
        CHECK(approx(sf.evaluate(u), 5.0));
        sf.add_context("3", std::make_shared<Context>("a", "aa"));
        CHECK(approx(sf.evaluate(u), 9.0));
        EvaluatedScoreFunction table;
        sf.evaluate(u, table);
        CHECK(table.size() == 3 && table[0].name == "1: " && table[2].term == 4.0);
    }
}

static void test_macrostate_prob_term() {
    auto dev = std::make_shared<Device>("");
    dev->add_macrostate("dummy", "");
    struct T {
        string name;
        ConditionEnum c;
        FavorableEnum f;
        double apo, holo, expect;
    };
    using C = ConditionEnum;
    using F = FavorableEnum;
    const std::vector<T> tests = {
        {"apo: not dummy", C::APO, F::NO, 0.2, 0.2, std::log(0.8)},
        {"apo: not dummy", C::APO, F::NO, 0.9, 0.2, std::log(0.1)},
        {"apo: not dummy", C::APO, F::NO, 0.2, 0.9, std::log(0.8)},
        {"apo: not dummy", C::APO, F::NO, 0.9, 0.9, std::log(0.1)},
        {"apo: dummy", C::APO, F::YES, 0.2, 0.2, std::log(0.2)},
        {"apo: dummy", C::APO, F::YES, 0.9, 0.2, std::log(0.9)},
        {"apo: dummy", C::APO, F::YES, 0.2, 0.9, std::log(0.2)},
        {"apo: dummy", C::APO, F::YES, 0.9, 0.9, std::log(0.9)},
        {"holo: not dummy", C::HOLO, F::NO, 0.2, 0.2, std::log(0.8)},
        {"holo: not dummy", C::HOLO, F::NO, 0.9, 0.2, std::log(0.8)},
        {"holo: not dummy", C::HOLO, F::NO, 0.2, 0.9, std::log(0.1)},
        {"holo: not dummy", C::HOLO, F::NO, 0.9, 0.9, std::log(0.1)},
        {"holo: dummy", C::HOLO, F::YES, 0.2, 0.2, std::log(0.2)},
        {"holo: dummy", C::HOLO, F::YES, 0.9, 0.2, std::log(0.2)},
        {"holo: dummy", C::HOLO, F::YES, 0.2, 0.9, std::log(0.9)},
        {"holo: dummy", C::HOLO, F::YES, 0.9, 0.9, std::log(0.9)},
    };
    for (auto &t : tests) {
        DummyRnaFold apo(t.apo), holo(t.holo);
        MacrostateProbTerm term("dummy", t.c, t.f);
        CHECK(term.name() == t.name);
        CHECK(approx(term.evaluate(dev, apo, holo), t.expect));
    }
}

// ------------------------------------------------------------ config + TSV
static void test_yaml_and_config() {
    const char *cfg =
        "# addapt config\n"
        "sequence: 'ACGUacguNNNN'\n"
        "macrostates:\n"
        "  active: \"((..))......\"\n"
        "  other:  '....xx......'   # comment\n"
        "objective:\n"
        "  apo: not active\n"
        "  holo: active\n"
        "aptamer:\n"
        "  sequence: GAUACCAGCCGAAAGGCCCUUGGCAGC\n"
        "  fold: (...((.(((....)))....))...)\n"
        "  affinity: 0.32\n"
        "contexts:\n"
        "  gfp: [GG, 'CC']\n"
        "  none:\n"
        "    - ''\n"
        "    - ''\n"
        "thermostat: 5 to 0 in 300 steps\n";
    yaml::Node n = yaml::parse(cfg);
    CHECK(n["sequence"].as_string() == "ACGUacguNNNN");
    CHECK(n["macrostates"]["other"].as_string() == "....xx......");
    CHECK(n["contexts"]["gfp"][1].as_string() == "CC");
    CHECK(n["contexts"]["none"][0].as_string() == "");
    CHECK(n["aptamer"]["fold"].as_string() == "(...((.(((....)))....))...)");
    CHECK(!n["missing"]);
    CHECK_THROWS(yaml::parse("a: 1\n  b: 2\n"));
    CHECK_THROWS(yaml::parse("a: 1\na: 2\n"));
    const string path = "/tmp/adx_test_cfg.yml", path2 = "/tmp/adx_test_cfg2.yml";
    { std::ofstream f(path); f << cfg; }
    auto dev = device_from_yaml({path});
    CHECK(dev->seq() == "ACGUacguNNNN" && dev->macrostate("active") == "((..))......");
    auto sf = scorefxn_from_yaml({path});
    CHECK(sf->terms().size() == 2 && sf->terms()[0]->name() == "apo: not active" && sf->terms()[1]->name() == "holo: active");
    CHECK(sf->aptamer() && approx(sf->aptamer()->affinity(), 0.32));
    CHECK(sf->contexts().size() == 2 && sf->context("gfp")->before() == "GG" && sf->context("gfp")->after() == "CC");
    auto th = std::dynamic_pointer_cast<AnnealingThermostat>(thermostat_from_yaml({path}));
    CHECK(th && th->cycle_len() == 300);
    { std::ofstream f(path2); f << "sequence: ACGU\n"; }
    CHECK_THROWS(device_from_yaml({path, path2}));   // 2 'sequence' sections
    CHECK_THROWS(score_term_from_str(ConditionEnum::APO, "not a macrostate"));
    auto t = std::dynamic_pointer_cast<MacrostateProbTerm>(score_term_from_str(ConditionEnum::HOLO, "not x1"));
    CHECK(t && t->macrostate() == "x1" && t->favorable() == FavorableEnum::NO);
}

static void test_reference_loop_and_tsv() {
    // the reference loop over dummy folds: every proposal scores 0 (ln 0.5 * 2
    // terms is constant), so every changed step is ACCEPT_WORSENED at T = 1
    auto dev = std::make_shared<Device>("NNNNNNNNNN");
    dev->add_macrostate("active", "((......))");
    auto sf = std::make_shared<ScoreFunction>();
    sf->fold_factory(dummy_factory);
    *sf += std::make_shared<MacrostateProbTerm>("active", ConditionEnum::APO, FavorableEnum::NO);
    *sf += std::make_shared<MacrostateProbTerm>("active", ConditionEnum::HOLO);
    MonteCarlo mc;
    mc += std::make_shared<UnbiasedMutationMove>();
    mc.scorefxn(sf);
    mc.num_steps(20);
    const string path = "/tmp/adx_test_traj.tsv";
    mc += std::make_shared<TsvTrajectoryReporter>(path, 2);
    std::mt19937 rng(0);
    DevicePtr out = mc.apply(dev, rng);
    CHECK(out->seq() != dev->seq());
    std::ifstream f(path);
    std::string line;
    std::vector<string> lines;
    while (std::getline(f, line)) lines.push_back(line);
    CHECK(lines.size() == 2 + 10);
    CHECK(lines[0] == "#\tinitial_seq\tNNNNNNNNNN");
    CHECK(lines[1].rfind("step\tnum_steps\tcurrent_score\tproposed_score\tterm_weight[apo: not active]\t"
                         "term_value[apo: not active]\tterm_weight[holo: active]\tterm_value[holo: active]\t"
                         "score_diff\ttemperature\tmetropolis_criterion\trandom_threshold\tmove\toutcome\t"
                         "current_seq\tproposed_seq", 0) == 0);
    CHECK(lines[2].rfind("0\t20\t", 0) == 0);
    CHECK(lines[2].find("UnbiasedMutation") != string::npos);
    // the partner rule held on every accepted sequence
    for (int k = 0; k < 2; k++) {
        const char a = out->seq()[k], b = out->seq()[9 - k];
        CHECK((a == 'N' && b == 'N') || (a != 'N' && COMPLEMENTARY_NUCS.at(a) == b));
    }
}

int main() {
    test_device();
    test_device_contexts();
    test_device_mutate();
    test_aptamer();
    test_mutable_positions();
    test_mutate_recursively();
    test_thermostats();
    test_score_function();
    test_macrostate_prob_term();
    test_yaml_and_config();
    test_reference_loop_and_tsv();
    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
