// Host-side energy model: ViennaRNA 2.0 parameter-file reader + loop energies.
// See energy.hpp.  The parameter sections and index conventions are those of
// ViennaRNA's write_parameter_file / read_parameter_file.
#include "energy.hpp"

#include <cctype>
#include <cmath>
#include <fstream>
#include <map>
#include <sstream>

namespace adx {

namespace {

const int PAIR_TABLE[5][5] = {{0, 0, 0, 0, 0},
                              {0, 0, 0, 0, 5},
                              {0, 0, 0, 1, 0},
                              {0, 0, 2, 0, 3},
                              {0, 6, 0, 4, 0}};
const int RTYPE_TABLE[8] = {0, 2, 1, 4, 3, 6, 5, 7};

struct Section {
    std::vector<double> values;
    std::vector<std::string> lines;
};

bool is_loop_section(const std::string &name) {
    return name == "Triloops" || name == "Tetraloops" || name == "Hexaloops";
}

}  // namespace

int base_code(char c) {
    switch (std::toupper(static_cast<unsigned char>(c))) {
    case 'A': return 1;
    case 'C': return 2;
    case 'G': return 3;
    case 'U':
    case 'T': return 4;
    default: return 0;
    }
}

int pair_type(int a, int b) { return PAIR_TABLE[a][b]; }
int rtype(int t) { return RTYPE_TABLE[t]; }

bool load_params(const std::string &path, EnergyParams &P, std::string &err) {
    std::ifstream in(path);
    if (!in) {
        err = "cannot open parameter file '" + path + "'";
        return false;
    }
    std::map<std::string, Section> secs;
    Section *cur = nullptr;
    std::string curname;
    std::string line;
    bool in_comment = false;
    while (std::getline(in, line)) {
        std::string s;
        for (size_t i = 0; i < line.size(); i++) {
            if (in_comment) {
                if (line[i] == '*' && i + 1 < line.size() && line[i + 1] == '/') {
                    in_comment = false;
                    i++;
                }
                continue;
            }
            if (line[i] == '/' && i + 1 < line.size() && line[i + 1] == '*') {
                in_comment = true;
                i++;
                continue;
            }
            s.push_back(line[i]);
        }
        size_t a = s.find_first_not_of(" \t\r\n");
        if (a == std::string::npos) continue;
        s = s.substr(a);
        if (s[0] == '#') {
            if (s.size() > 1 && s[1] == '#') continue;
            std::istringstream ss(s.substr(1));
            ss >> curname;
            if (curname == "END") break;
            cur = &secs[curname];
            continue;
        }
        if (!cur) continue;
        if (is_loop_section(curname)) {
            cur->lines.push_back(s);
            continue;
        }
        std::istringstream ss(s);
        std::string tok;
        while (ss >> tok) {
            if (tok == "INF") cur->values.push_back(INF_E);
            else if (tok == "DEF") cur->values.push_back(-50);
            else if (tok == "NST") cur->values.push_back(0);
            else {
                char *end = nullptr;
                double x = std::strtod(tok.c_str(), &end);
                if (end != tok.c_str()) cur->values.push_back(x);
            }
        }
    }
    auto need = [&](const char *name, size_t count) -> const std::vector<double> * {
        auto it = secs.find(name);
        if (it == secs.end()) {
            err = std::string("parameter file: missing section '") + name + "'";
            return nullptr;
        }
        if (it->second.values.size() < count) {
            err = std::string("parameter file: section '") + name + "' has " +
                  std::to_string(it->second.values.size()) + " values, need " +
                  std::to_string(count);
            return nullptr;
        }
        return &it->second.values;
    };
    auto iv = [](double x) { return static_cast<int>(std::lrint(x)); };
    const std::vector<double> *v;
    if (!(v = need("stack", 49))) return false;
    for (int a = 1; a <= 7; a++)
        for (int b = 1; b <= 7; b++) P.stack[a][b] = iv((*v)[(a - 1) * 7 + (b - 1)]);
    for (int a = 0; a < 8; a++) { P.stack[0][a] = INF_E; P.stack[a][0] = INF_E; }
    struct MM { const char *name; int (*t)[5][5]; } mms[] = {
        {"mismatch_hairpin", P.mmH},       {"mismatch_interior", P.mmI},
        {"mismatch_interior_1n", P.mm1nI}, {"mismatch_interior_23", P.mm23I},
        {"mismatch_multi", P.mmM},         {"mismatch_exterior", P.mmExt}};
    for (auto &m : mms) {
        if (!(v = need(m.name, 175))) return false;
        for (int x = 0; x < 5; x++)
            for (int y = 0; y < 5; y++) m.t[0][x][y] = INF_E;
        for (int a = 1; a <= 7; a++)
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++) m.t[a][x][y] = iv((*v)[(a - 1) * 25 + x * 5 + y]);
    }
    if (!(v = need("dangle5", 35))) return false;
    for (int a = 1; a <= 7; a++)
        for (int x = 0; x < 5; x++) P.d5[a][x] = iv((*v)[(a - 1) * 5 + x]);
    if (!(v = need("dangle3", 35))) return false;
    for (int a = 1; a <= 7; a++)
        for (int x = 0; x < 5; x++) P.d3[a][x] = iv((*v)[(a - 1) * 5 + x]);
    for (int x = 0; x < 5; x++) { P.d5[0][x] = INF_E; P.d3[0][x] = INF_E; }
    if (!(v = need("int11", 49 * 25))) return false;
    for (int a = 0; a < 8; a++)
        for (int b = 0; b < 8; b++)
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++)
                    P.int11[a][b][x][y] =
                        (a && b) ? iv((*v)[((a - 1) * 7 + (b - 1)) * 25 + x * 5 + y]) : INF_E;
    if (!(v = need("int21", 49 * 125))) return false;
    for (int a = 0; a < 8; a++)
        for (int b = 0; b < 8; b++)
            for (int x = 0; x < 5; x++)
                for (int y = 0; y < 5; y++)
                    for (int z = 0; z < 5; z++)
                        P.int21[a][b][x][y][z] =
                            (a && b) ? iv((*v)[((a - 1) * 7 + (b - 1)) * 125 + x * 25 + y * 5 + z])
                                     : INF_E;
    if (!(v = need("int22", 36 * 256))) return false;
    for (int a = 0; a < 8; a++)
        for (int b = 0; b < 8; b++)
            for (int w = 0; w < 5; w++)
                for (int x = 0; x < 5; x++)
                    for (int y = 0; y < 5; y++)
                        for (int z = 0; z < 5; z++) {
                            bool in = a >= 1 && a <= 6 && b >= 1 && b <= 6 && w && x && y && z;
                            P.int22[a][b][w][x][y][z] =
                                in ? iv((*v)[((a - 1) * 6 + (b - 1)) * 256 + (w - 1) * 64 +
                                             (x - 1) * 16 + (y - 1) * 4 + (z - 1)])
                                   : INF_E;
                        }
    if (!(v = need("hairpin", 31))) return false;
    for (int i = 0; i < 31; i++) P.hairpin[i] = iv((*v)[i]);
    if (!(v = need("bulge", 31))) return false;
    for (int i = 0; i < 31; i++) P.bulge[i] = iv((*v)[i]);
    if (!(v = need("interior", 31))) return false;
    for (int i = 0; i < 31; i++) P.interior[i] = iv((*v)[i]);
    if (!(v = need("ML_params", 6))) return false;
    P.MLbase = iv((*v)[0]);
    P.MLclosing = iv((*v)[2]);
    P.MLintern = iv((*v)[4]);
    if (!(v = need("NINIO", 3))) return false;
    P.ninio = iv((*v)[0]);
    P.maxninio = iv((*v)[2]);
    if (!(v = need("Misc", 5))) return false;
    P.DuplexInit = iv((*v)[0]);
    P.TermAU = iv((*v)[2]);
    P.lxc = (*v)[4];
    struct L { const char *name; size_t len; std::vector<std::pair<std::string, int>> *out; } loops[] = {
        {"Triloops", 5, &P.triloops}, {"Tetraloops", 6, &P.tetraloops}, {"Hexaloops", 8, &P.hexaloops}};
    for (auto &l : loops) {
        l.out->clear();
        auto it = secs.find(l.name);
        if (it == secs.end()) continue;
        for (auto &ln : it->second.lines) {
            std::istringstream ss(ln);
            std::string sq;
            int e;
            if ((ss >> sq >> e) && sq.size() == l.len) l.out->push_back({sq, e});
        }
    }
    return true;
}

double hairpin_energy(const EnergyParams &P, const std::vector<int> &S, const std::string &useq,
                      int i, int j) {
    int u = j - i - 1;
    int type = pair_type(S[i], S[j]);
    double e = (u <= 30) ? P.hairpin[u] : P.hairpin[30] + P.lxc * std::log(u / 30.0);
    if (u < 3) return e;
    auto match = [&](const std::vector<std::pair<std::string, int>> &tab, int len, int &out) {
        for (auto &t : tab)
            if (useq.compare(i, len, t.first) == 0) { out = t.second; return true; }
        return false;
    };
    int sp;
    if (u == 4 && match(P.tetraloops, 6, sp)) return sp;
    if (u == 6 && match(P.hexaloops, 8, sp)) return sp;
    if (u == 3) {
        if (match(P.triloops, 5, sp)) return sp;
        return e + (type > 2 ? P.TermAU : 0);
    }
    return e + P.mmH[type][S[i + 1]][S[j - 1]];
}

double interior_energy(const EnergyParams &P, int n1, int n2, int type, int type2, int si1,
                       int sj1, int sp1, int sq1) {
    int nl = std::max(n1, n2), ns = std::min(n1, n2);
    double e;
    if (nl == 0) return P.stack[type][type2];
    if (ns == 0) {
        e = (nl <= MAXLOOP) ? P.bulge[nl] : P.bulge[30] + P.lxc * std::log(nl / 30.0);
        if (nl == 1) e += P.stack[type][type2];
        else {
            if (type > 2) e += P.TermAU;
            if (type2 > 2) e += P.TermAU;
        }
        return e;
    }
    if (ns == 1) {
        if (nl == 1) return P.int11[type][type2][si1][sj1];
        if (nl == 2) {
            if (n1 == 1) return P.int21[type][type2][si1][sq1][sj1];
            return P.int21[type2][type][sq1][si1][sp1];
        }
        e = (nl + 1 <= MAXLOOP) ? P.interior[nl + 1]
                                : P.interior[30] + P.lxc * std::log((nl + 1) / 30.0);
        e += std::min(P.maxninio, (nl - ns) * P.ninio);
        e += P.mm1nI[type][si1][sj1] + P.mm1nI[type2][sq1][sp1];
        return e;
    }
    if (ns == 2) {
        if (nl == 2) return P.int22[type][type2][si1][sp1][sq1][sj1];
        if (nl == 3) {
            e = P.interior[5] + P.ninio;
            e += P.mm23I[type][si1][sj1] + P.mm23I[type2][sq1][sp1];
            return e;
        }
    }
    int u = nl + ns;
    e = (u <= MAXLOOP) ? P.interior[u] : P.interior[30] + P.lxc * std::log(u / 30.0);
    e += std::min(P.maxninio, (nl - ns) * P.ninio);
    e += P.mmI[type][si1][sj1] + P.mmI[type2][sq1][sp1];
    return e;
}

int ext_stem_energy(const EnergyParams &P, int type, int n5d, int n3d) {
    int e = 0;
    if (n5d >= 0 && n3d >= 0) e += P.mmExt[type][n5d][n3d];
    else if (n5d >= 0) e += P.d5[type][n5d];
    else if (n3d >= 0) e += P.d3[type][n3d];
    if (type > 2) e += P.TermAU;
    return e;
}

int ml_stem_energy(const EnergyParams &P, int type, int n5d, int n3d) {
    int e = 0;
    if (n5d >= 0 && n3d >= 0) e += P.mmM[type][n5d][n3d];
    else if (n5d >= 0) e += P.d5[type][n5d];
    else if (n3d >= 0) e += P.d3[type][n3d];
    if (type > 2) e += P.TermAU;
    return e + P.MLintern;
}

double eval_structure(const EnergyParams &P, const std::string &seq, const std::string &st) {
    const int N = static_cast<int>(seq.size());
    if (static_cast<int>(st.size()) != N) return NAN;
    std::vector<int> S(N + 2, 0), pt(N + 2, 0), stk;
    std::string useq(N + 2, ' ');
    for (int i = 1; i <= N; i++) {
        S[i] = base_code(seq[i - 1]);
        char c = static_cast<char>(std::toupper(static_cast<unsigned char>(seq[i - 1])));
        useq[i] = (c == 'T') ? 'U' : c;
    }
    if (N) { S[0] = S[N]; S[N + 1] = S[1]; }
    for (int i = 1; i <= N; i++) {
        if (st[i - 1] == '(') stk.push_back(i);
        else if (st[i - 1] == ')') {
            if (stk.empty()) return NAN;
            int a = stk.back();
            stk.pop_back();
            pt[a] = i;
            pt[i] = a;
        }
    }
    if (!stk.empty()) return NAN;
    double e = 0.0;
    for (int i = 1; i <= N; i++) {
        if (pt[i] > i) {
            int j = pt[i];
            e += ext_stem_energy(P, pair_type(S[i], S[j]), i > 1 ? S[i - 1] : -1, j < N ? S[j + 1] : -1);
            i = j;
        }
    }
    for (int i = 1; i <= N; i++) {
        int j = pt[i];
        if (j <= i) continue;
        int type = pair_type(S[i], S[j]);
        if (!type) return NAN;
        int nb = 0, p = 0, q = 0, unp = 0;
        double ml = 0.0;
        for (int k = i + 1; k < j; k++) {
            if (pt[k] > k) {
                if (++nb == 1) { p = k; q = pt[k]; }
                ml += ml_stem_energy(P, pair_type(S[k], S[pt[k]]), S[k - 1], S[pt[k] + 1]);
                k = pt[k];
            } else {
                unp++;
            }
        }
        if (nb == 0) e += hairpin_energy(P, S, useq, i, j);
        else if (nb == 1) {
            int type2 = pair_type(S[q], S[p]);
            if (!type2) return NAN;
            e += interior_energy(P, p - i - 1, j - q - 1, type, type2, S[i + 1], S[j - 1], S[p - 1],
                                 S[q + 1]);
        } else {
            e += P.MLclosing + ml_stem_energy(P, rtype(type), S[j - 1], S[i + 1]) + ml +
                 unp * P.MLbase;
        }
    }
    return e / 100.0;
}

}  // namespace adx
