// Host-side nearest-neighbour energy model for the MI355X engine.
//
// Reads a ViennaRNA 2.0 parameter file (the model ViennaRNA's
// vrna_md_set_default selects in /root/reference/src/scoring.cc:80-83) and
// turns it into the FP32 Boltzmann tables the gfx950 kernels read from HBM
// (DevParams).  Also evaluates the free energy of a single structure, which
// the ligand-motif soft constraint needs (scoring.cc:92-100).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace adx {

constexpr int INF_E = 10000000;
constexpr int MAXLOOP = 30;
constexpr int TURN = 3;
constexpr double GASCONST = 1.98717;  // cal/(mol K)
constexpr double K0 = 273.15;
constexpr double TEMPERATURE = 37.0;

inline double kT_cal() { return (TEMPERATURE + K0) * GASCONST; }
inline double kT_kcal() { return kT_cal() / 1000.0; }

// Integer (dcal/mol) parameter set, ViennaRNA indexing: pair types 1..7
// (CG GC GU UG AU UA NS), bases 0..4 (N A C G U).
struct EnergyParams {
    int stack[8][8];
    int mmH[8][5][5], mmI[8][5][5], mm1nI[8][5][5], mm23I[8][5][5], mmM[8][5][5], mmExt[8][5][5];
    int d5[8][5], d3[8][5];
    int int11[8][8][5][5];
    int int21[8][8][5][5][5];
    int int22[8][8][5][5][5][5];
    int hairpin[31], bulge[31], interior[31];
    int MLbase, MLclosing, MLintern;
    int ninio, maxninio, TermAU, DuplexInit;
    double lxc;
    std::vector<std::pair<std::string, int>> triloops, tetraloops, hexaloops;
};

// Parse; returns false and fills err on failure.
bool load_params(const std::string &path, EnergyParams &P, std::string &err);

int base_code(char c);                 // ACGU(T) -> 1..4, else 0 (N)
int pair_type(int a, int b);           // 0 if not canonical
int rtype(int t);

// Loop energies (dcal/mol), ViennaRNA 2.x semantics with dangles = 2.
double hairpin_energy(const EnergyParams &P, const std::vector<int> &S, const std::string &useq,
                      int i, int j);  // 1-based, PF flavour (non-truncated lxc)
double interior_energy(const EnergyParams &P, int n1, int n2, int type, int type2, int si1,
                       int sj1, int sp1, int sq1);
int ext_stem_energy(const EnergyParams &P, int type, int n5d, int n3d);
int ml_stem_energy(const EnergyParams &P, int type, int n5d, int n3d);

// Free energy (kcal/mol) of `structure` on `seq`; NaN if malformed.
double eval_structure(const EnergyParams &P, const std::string &seq, const std::string &structure);

}  // namespace adx
