// Golden values of the RNG streams addapt draws from (sampling.cc:36-37, 65,
// 78, 298-300): std::mt19937, std::uniform_int_distribution<int> and
// std::generate_canonical<double, 53> as implemented by the libstdc++ the
// reference is built with.  Writes JSON to stdout.
#include <cstdio>
#include <random>

int main() {
    std::printf("{\n  \"generator\": \"g++ %d.%d libstdc++ %d\",\n", __GNUC__, __GNUC_MINOR__, _GLIBCXX_RELEASE);
    std::printf("  \"raw\": [");
    const unsigned seeds[] = {0u, 1u, 5489u, 1000u, 4095u};
    for (int s = 0; s < 5; s++) {
        std::mt19937 g(seeds[s]);
        std::printf("%s\n    {\"seed\": %u, \"out\": [", s ? "," : "", seeds[s]);
        for (int k = 0; k < 700; k++) std::printf("%s%u", k ? ", " : "", unsigned(g()));
        std::printf("]}");
    }
    std::printf("\n  ],\n  \"uniform_int\": [");
    const int his[] = {3, 9, 10, 25, 99, 1000000};
    int first = 1;
    for (int s = 0; s < 3; s++) {
        for (int h = 0; h < 6; h++) {
            std::mt19937 g(seeds[s]);
            std::uniform_int_distribution<int> d(0, his[h]);
            std::printf("%s\n    {\"seed\": %u, \"hi\": %d, \"out\": [", first ? "" : ",", seeds[s], his[h]);
            first = 0;
            for (int k = 0; k < 400; k++) std::printf("%s%d", k ? ", " : "", d(g));
            std::printf("]}");
        }
    }
    std::printf("\n  ],\n  \"canonical\": [");
    for (int s = 0; s < 3; s++) {
        std::mt19937 g(seeds[s]);
        std::printf("%s\n    {\"seed\": %u, \"out\": [", s ? "," : "", seeds[s]);
        for (int k = 0; k < 400; k++) std::printf("%s%.17g", k ? ", " : "", std::generate_canonical<double, 53>(g));
        std::printf("]}");
    }
    std::printf("\n  ]\n}\n");
    return 0;
}
