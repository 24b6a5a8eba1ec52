// GpuRnaFold::base_pair_prob (the C++ host mirror of ViennaRnaFold,
// scoring.cc:37-51) on the GPU: prints "i j p" for every i < j of the
// given sequence, optionally in the holo fold of the THEO aptamer.
// usage: bpp_probe <seq> [holo]
#include <cstdio>
#include <memory>
#include <string>

#include "addapt/model.hh"
#include "addapt/scoring.hh"

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    try {
        auto dev = std::make_shared<addapt::Device>(argv[1]);
        addapt::AptamerConstPtr apt;
        if (argc > 2 && std::string(argv[2]) == "holo")
            apt = std::make_shared<addapt::Aptamer>("GAUACCAGCCGAAAGGCCCUUGGCAGC", "(...((.(((....)))....))...)", 0.32);
        addapt::ViennaRnaFold fold(dev, apt);
        const int n = static_cast<int>(std::string(argv[1]).size());
        for (int i = 0; i < n; i++)
            for (int j = i + 1; j < n; j++) std::printf("%d %d %.9g\n", i, j, fold.base_pair_prob(i, j));
        std::printf("sym %.9g\n", fold.base_pair_prob(n - 1, 0));
    } catch (std::string &e) {
        std::fprintf(stderr, "Error: %s\n", e.c_str());
        return 1;
    }
    return 0;
}
