// addapt: Monte Carlo sgRNA design from config files (the reference's
// apps/addapt.cc command line, run on the MI355X engine).
//
//   addapt <config>... [-n <num>] [-T <schedule>] [-r <seed>] [-o <path>]
//                      [-i <steps>] [--walkers <W>] [--gpu <id>] [--params <file>]
//                      [--reference-loop]
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "addapt/config.hh"
#include "addapt/model.hh"
#include "addapt/sampling.hh"
#include "addapt/scoring.hh"

using namespace addapt;

static const char USAGE[] =
    "Run a Monte Carlo design simulation of an sgRNA with an aptamer (addapt).\n"
    "\n"
    "Usage:\n"
    "  addapt <config>... [options]\n"
    "\n"
    "Options:\n"
    "  -n <num>, --num-moves <num>            [default: 100]\n"
    "    The number of moves to attempt in the design simulation.\n"
    "  -T <schedule>, --temperature <schedule>\n"
    "    Metropolis temperature: fixed (\"5\"), annealing (\"1 to 0 in 500 steps\")\n"
    "    or auto-scaling (\"auto 50%\").  Default: the config's 'thermostat' or 1.\n"
    "  -r <seed>, --random-seed <seed>        [default: 0]\n"
    "    Seed of the random number generator (std::mt19937).\n"
    "  -o <path>, --output <path>             [default: traj.tsv]\n"
    "    Trajectory (TSV) of the simulation.\n"
    "  -i <steps>, --output-interval <steps>  [default: 1]\n"
    "    How often a snapshot is recorded.\n"
    "  --walkers <W>                          [default: 1]\n"
    "    Run W independent walkers (seeds r .. r+W-1) on the GPU at once and write\n"
    "    their final sequences and scores to the output instead of a trajectory.\n"
    "  --gpu <id>                             [default: 0]\n"
    "  --params <file>  Energy parameters (ViennaRNA 2.0 format).\n"
    "  --reference-loop  Run the reference's single-walker loop (one GPU fold call\n"
    "    per partition function) instead of the fused engine.\n"
    "  --version\n"
    "  -h, --help\n";

int main(int argc, char **argv) {
    std::vector<std::string> configs;
    std::string temp, out = "traj.tsv", params;
    int num = 100, interval = 1, walkers = 1, gpu = 0;
    unsigned long seed = 0;
    bool ref_loop = false;
    try {
        for (int k = 1; k < argc; k++) {
            const std::string a = argv[k];
            auto val = [&](const char *name) -> std::string {
                if (k + 1 >= argc) throw std::string("option ") + name + " needs a value";
                return argv[++k];
            };
            if (a == "-h" || a == "--help") { std::cout << USAGE; return 0; }
            else if (a == "--version") { std::cout << "addapt-amd 0.1\n"; return 0; }
            else if (a == "-n" || a == "--num-moves") num = std::stoi(val("--num-moves"));
            else if (a == "-T" || a == "--temperature") temp = val("--temperature");
            else if (a == "-r" || a == "--random-seed") seed = std::stoul(val("--random-seed"));
            else if (a == "-o" || a == "--output") out = val("--output");
            else if (a == "-i" || a == "--output-interval") interval = std::stoi(val("--output-interval"));
            else if (a == "--walkers") walkers = std::stoi(val("--walkers"));
            else if (a == "--gpu") gpu = std::stoi(val("--gpu"));
            else if (a == "--params") params = val("--params");
            else if (a == "--reference-loop") ref_loop = true;
            else if (!a.empty() && a[0] == '-') throw std::string("unknown option '" + a + "'");
            else configs.push_back(a);
        }
        if (configs.empty()) {
            std::cerr << USAGE;
            return 1;
        }
        if (!params.empty()) set_parameter_file(params);
        DevicePtr device = device_from_yaml(configs);
        ScoreFunctionPtr sf = scorefxn_from_yaml(configs);
        auto mc = std::make_shared<MonteCarlo>();
        *mc += std::make_shared<UnbiasedMutationMove>();
        mc->thermostat(!temp.empty() ? thermostat_from_str(temp) : thermostat_from_yaml(configs));
        mc->num_steps(num);
        mc->scorefxn(sf);
        mc->gpu(gpu);
        if (walkers > 1) {
            std::vector<uint32_t> seeds(walkers);
            for (int w = 0; w < walkers; w++) seeds[w] = uint32_t(seed + w);
            auto res = mc->apply_batch(device, seeds, gpu);
            FILE *f = std::fopen(out.c_str(), "w");
            if (!f) throw std::string("couldn't open '" + out + "' for writing");
            std::fprintf(f, "walker\tseed\tscore\treject\taccept_worsened\taccept_unchanged\taccept_improved\tseq\n");
            for (int w = 0; w < walkers; w++) {
                auto &c = res[w].outcome_counters;
                std::fprintf(f, "%d\t%u\t%.17g\t%lld\t%lld\t%lld\t%lld\t%s\n", w, seeds[w], res[w].score,
                             c[OutcomeEnum::REJECT], c[OutcomeEnum::ACCEPT_WORSENED],
                             c[OutcomeEnum::ACCEPT_UNCHANGED], c[OutcomeEnum::ACCEPT_IMPROVED],
                             res[w].device->seq().c_str());
            }
            std::fclose(f);
            return 0;
        }
        *mc += std::make_shared<ProgressReporter>();
        *mc += std::make_shared<TsvTrajectoryReporter>(out, interval);
        if (ref_loop) {
            std::mt19937 rng(static_cast<uint32_t>(seed));
            mc->apply(device, rng);
        } else {
            mc->apply(device, static_cast<uint32_t>(seed));
        }
        return 0;
    } catch (const std::string &e) {
        std::cerr << "Error: " << e << std::endl;
        return 1;
    } catch (const char *e) {
        std::cerr << "Error: " << e << std::endl;
        return 1;
    } catch (const std::exception &e) {
        std::cerr << "Error: " << e.what() << std::endl;
        return 1;
    }
}
