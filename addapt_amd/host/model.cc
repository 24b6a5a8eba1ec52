// Device / Aptamer / Context (reference src/model.cc semantics).
#include "addapt/model.hh"

#include <cstdio>

namespace addapt {

static string fmt_err(const char *f, int a, int b) {
    char buf[160];
    std::snprintf(buf, sizeof buf, f, a, b);
    return buf;
}

Context::Context(string before, string after) : before_(before), after_(after) {}

Aptamer::Aptamer(string seq, string fold, double affinity_uM) : seq_(seq), fold_(fold), affinity_(affinity_uM) {}

Device::Device(string seq) : seq_(seq), context_(std::make_shared<Context>()) {}

int Device::index(int i, int n) const {
    const int k = i < 0 ? n + i : i;
    if (k < 0 || k >= n) throw fmt_err("index %d out of range for a sequence of length %d", i, n);
    return k;
}

int Device::len() const { return static_cast<int>(context_->before().size() + seq_.size() + context_->after().size()); }

string Device::seq() const { return context_->before() + seq_ + context_->after(); }

char Device::seq(int i) const { return seq()[index(i, len())]; }

char Device::raw_seq(int i) const { return seq_[index(i, raw_len())]; }

string Device::macrostate(string name) const {
    auto it = macro_.find(name);
    if (it == macro_.end()) throw string("no macrostate named '" + name + "'");
    return string(context_->before().size(), '.') + it->second + string(context_->after().size(), '.');
}

// model.cc:59-64 (the reference throws a const char* here; std::string is what
// its callers catch, so that is what this mirror throws)
void Device::add_macrostate(string name, string constraint) {
    if (constraint.size() != seq_.size()) throw string("constraint length doesn't match sequence length");
    macro_[name] = constraint;
}

std::vector<std::pair<string, string>> Device::macrostates() const {
    std::vector<std::pair<string, string>> out;
    for (auto &kv : macro_) out.emplace_back(kv.first, macrostate(kv.first));
    return out;
}

std::vector<string> Device::macrostate_names() const {
    std::vector<string> out;
    for (auto &kv : macro_) out.push_back(kv.first);
    return out;
}

void Device::context(ContextConstPtr c) { context_ = c ? c : std::make_shared<Context>(); }

void Device::remove_context() { context_ = std::make_shared<Context>(); }

void Device::mutate(int i, char base) { seq_[index(i, raw_len())] = base; }

DevicePtr Device::copy() const { return std::make_shared<Device>(*this); }

void Device::assign(DeviceConstPtr other) { *this = *other; }

}  // namespace addapt
