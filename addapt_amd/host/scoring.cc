// Folding and scoring (reference src/scoring.cc semantics), folds on the GPU.
#include "addapt/scoring.hh"

#include <dlfcn.h>

#include <cmath>
#include <cstdlib>
#include <mutex>
#include <ostream>

#include "gpu.hh"

namespace addapt {
namespace gpu {

namespace {
std::string g_path;
adx_params *g_params = nullptr;
std::mutex g_mu;

// ADX_PARAMS, else addapt_amd/data/ next to this library (addapt_amd/_lib/)
std::string default_path() {
    if (const char *e = std::getenv("ADX_PARAMS")) return e;
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&default_path), &info) && info.dli_fname) {
        std::string lib = info.dli_fname;
        const size_t slash = lib.rfind('/');
        const std::string dir = slash == std::string::npos ? "." : lib.substr(0, slash);
        return dir + "/../data/rna_turner2004_addapt.par";
    }
    return "addapt_amd/data/rna_turner2004_addapt.par";
}
}  // namespace

const adx_params *params() {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_params) {
        if (g_path.empty()) g_path = default_path();
        check(adx_params_load(g_path.c_str(), &g_params));
    }
    return g_params;
}

void set_params_path(const std::string &path) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_params) adx_params_free(g_params);
    g_params = nullptr;
    g_path = path;
}

}  // namespace gpu

void set_parameter_file(const string &path) { gpu::set_params_path(path); }

double kT() { return adx_kT(); }

// ---------------------------------------------------------------- GpuRnaFold
GpuRnaFold::GpuRnaFold(DeviceConstPtr device, AptamerConstPtr aptamer, int g)
    : seq_(device->seq()), aptamer_(aptamer), gpu_(g) {}

// scoring.cc:53-71: Z without and with the macrostate's hard constraint
double GpuRnaFold::macrostate_prob(string constraint) const {
    adx_fold *raw = nullptr;
    gpu::check(adx_fold_create(gpu::params(), seq_.c_str(), 0, gpu_, &raw));
    gpu::FoldPtr f(raw);
    if (aptamer_)
        gpu::check(adx_fold_add_motif(f.get(), aptamer_->seq().c_str(), aptamer_->fold().c_str(),
                                      kT() * std::log(aptamer_->affinity() / 1e6)));
    float g_tot = 0.f, g_act = 0.f;
    gpu::check(adx_fold_pf(f.get(), &g_tot));
    gpu::check(adx_fold_add_constraint(f.get(), constraint.c_str()));
    gpu::check(adx_fold_pf(f.get(), &g_act));
    return std::exp((double(g_tot) - double(g_act)) / kT());
}

// scoring.cc:37-51 (0-based, symmetric)
double GpuRnaFold::base_pair_prob(int i, int j) const {
    const int n = static_cast<int>(seq_.size());
    if (i < 0 || j < 0 || i >= n || j >= n) throw string("base pair index out of range");
    if (i == j) return 0.0;
    if (!bppm_fold_) {
        adx_fold *raw = nullptr;
        gpu::check(adx_fold_create(gpu::params(), seq_.c_str(), 1, gpu_, &raw));
        std::shared_ptr<::adx_fold> f(raw, adx_fold_free);
        if (aptamer_)
            gpu::check(adx_fold_add_motif(f.get(), aptamer_->seq().c_str(), aptamer_->fold().c_str(),
                                          kT() * std::log(aptamer_->affinity() / 1e6)));
        bppm_fold_ = f;
    }
    double p = 0.0;   // the matrix is computed on the first call and cached by the fold
    gpu::check(adx_fold_bpp(bppm_fold_.get(), std::min(i, j) + 1, std::max(i, j) + 1, &p));
    return p;
}

// ---------------------------------------------------------------- terms
static string term_name(ConditionEnum c, FavorableEnum f, const string &m) {
    return string(c == ConditionEnum::APO ? "apo: " : "holo: ") + (f == FavorableEnum::NO ? "not " : "") + m;
}

MacrostateProbTerm::MacrostateProbTerm(string macrostate, ConditionEnum cond, FavorableEnum fav)
    : ScoreTerm(term_name(cond, fav, macrostate), 1.0), macrostate_(macrostate), condition_(cond), favorable_(fav) {}

double MacrostateProbTerm::evaluate(DeviceConstPtr device, RnaFold const &apo, RnaFold const &holo) const {
    RnaFold const &fold = condition_ == ConditionEnum::APO ? apo : holo;
    double p = fold.macrostate_prob(device->macrostate(macrostate_));
    if (favorable_ == FavorableEnum::NO) p = 1.0 - p;
    return std::log(p);
}

// ---------------------------------------------------------------- score function
static std::shared_ptr<RnaFold> gpu_fold(DeviceConstPtr d, AptamerConstPtr a) {
    return std::make_shared<GpuRnaFold>(d, a);
}

ScoreFunction::ScoreFunction() : factory_(gpu_fold) {}

double ScoreFunction::evaluate(DeviceConstPtr device) const {
    EvaluatedScoreFunction table;
    return evaluate(device, table);
}

// scoring.cc:114-138: once, or once per context in name order with "name: " prefixes
double ScoreFunction::evaluate(DeviceConstPtr device, EvaluatedScoreFunction &table) const {
    table.clear();
    if (contexts_.empty()) return evaluate_terms(device, table);
    double score = 0.0;
    DevicePtr scratch = device->copy();
    for (auto &kv : contexts_) {
        scratch->context(kv.second);
        score += evaluate_terms(scratch, table, kv.first + ": ");
    }
    return score;
}

double ScoreFunction::evaluate_terms(DeviceConstPtr device, EvaluatedScoreFunction &table, string prefix) const {
    auto apo = factory_(device, nullptr);
    auto holo = factory_(device, aptamer_);
    double score = 0.0;
    for (auto &t : terms_) {
        EvaluatedScoreTerm e{prefix + t->name(), t->weight(), t->evaluate(device, *apo, *holo)};
        table.push_back(e);
        score += e.weight * e.term;
    }
    return score;
}

ContextConstPtr ScoreFunction::context(string name) const {
    auto it = contexts_.find(name);
    if (it == contexts_.end()) throw string("no context named '" + name + "'");
    return it->second;
}

}  // namespace addapt

namespace std {
ostream &operator<<(ostream &out, const addapt::ConditionEnum &c) {
    return out << (c == addapt::ConditionEnum::APO ? "APO" : "HOLO");
}
ostream &operator<<(ostream &out, const addapt::FavorableEnum &f) {
    return out << (f == addapt::FavorableEnum::YES ? "FAVORABLE" : "UNFAVORABLE");
}
}  // namespace std
