// Golden vectors for AutoScalingThermostat's median (reference sampling.cc:
// 389-396): std::nth_element(begin, begin + n/2, end) over doubles and the
// std::max(t, 0.0) clamp, run with the host libstdc++.  Arrays mix ties,
// +0.0 / -0.0, NaN and (for the depth-limit / heap_select path) adversarial
// orders.  Values are written as IEEE-754 bit patterns (hex) so signed zeros
// and NaN survive JSON.
#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

static uint64_t bits(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }

static void emit(const std::vector<double> &in, bool last) {
    std::vector<double> a(in);
    const size_t k = a.size() / 2;
    std::nth_element(a.begin(), a.begin() + k, a.end());
    const double t = std::max(a[k] / std::log(0.5), 0.0);
    std::printf("    {\"in\": [");
    for (size_t i = 0; i < in.size(); i++) std::printf("%s\"%016" PRIx64 "\"", i ? ", " : "", bits(in[i]));
    std::printf("], \"out\": [");
    for (size_t i = 0; i < a.size(); i++) std::printf("%s\"%016" PRIx64 "\"", i ? ", " : "", bits(a[i]));
    std::printf("], \"k\": %zu, \"T_rate_0.5\": \"%016" PRIx64 "\"}%s\n", k, bits(t), last ? "" : ",");
}

int main() {
    std::mt19937 g(20261017);
    std::vector<std::vector<double>> cases;
    const double pool[] = {0.0, -0.0, 0.25, -0.25, 1.5, -3.0, NAN, INFINITY, -INFINITY};
    for (int n : {1, 2, 3, 4, 5, 7, 8, 16, 17, 31, 64, 100, 257}) {
        for (int rep = 0; rep < 4; rep++) {
            std::vector<double> a(n);
            for (int i = 0; i < n; i++) {
                const unsigned r = g() % 16;
                if (rep == 0) a[i] = std::ldexp(double(int(g() % 2001) - 1000), -6);    // no specials
                else if (rep == 1) a[i] = r < 8 ? (r & 1 ? -0.0 : 0.0) : double(int(r) - 12);  // zeros
                else if (rep == 2) a[i] = pool[g() % 9];                                  // NaN / inf
                else a[i] = (g() % 5 == 0) ? NAN : std::ldexp(double(int(g() % 9) - 4), -2);
            }
            cases.push_back(a);
        }
    }
    // median-of-3 killer orders push introselect to its depth limit (heap_select)
    for (int n : {64, 200}) {
        std::vector<double> a(n);
        for (int i = 0; i < n; i++) a[i] = double(i % 2 ? n / 2 + i / 2 : i / 2);
        cases.push_back(a);
        std::vector<double> b(n);
        for (int i = 0; i < n; i++) b[i] = (i % 3 == 0) ? NAN : double((i * 7919) % 13) - 6.0;
        cases.push_back(b);
    }
    // a zero median with both signs present: which zero lands at k decides T's sign
    cases.push_back({0.0, -0.0, 0.0, -0.0, 0.0, 1.0, -1.0});
    cases.push_back({-0.0, 0.0, -0.0, 0.0, -0.0, 0.0, 2.0, -2.0, 0.0});
    std::printf("{\n  \"generator\": \"g++ 11.4 libstdc++ 11: std::nth_element + std::max(t, 0.0)\",\n  \"cases\": [\n");
    for (size_t c = 0; c < cases.size(); c++) emit(cases[c], c + 1 == cases.size());
    std::printf("  ]\n}\n");
}
