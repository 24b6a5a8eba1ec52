/* ViennaRNA 2.0 parameter-file reader for the oracle (test infrastructure).
 * Layout follows ViennaRNA's write_parameter_file (sections "# name", C
 * comments, INF/DEF tokens); the reference loads the same values implicitly
 * through vrna_md_set_default (/root/reference/src/scoring.cc:81). */
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "adx_oracle.h"

static char g_err[512];
const char *orc_last_error(void) { return g_err; }

double orc_kT_cal(void) { return (37.0 + 273.15) * 1.98717; }

typedef struct {
    char name[64];
    int n;
    int cap;
    double *v;           /* numeric tokens */
    int nlines;
    char (*lines)[64];   /* raw lines (special-loop sections) */
} section;

static void sec_push(section *s, double x) {
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 256;
        s->v = (double *)realloc(s->v, sizeof(double) * s->cap);
    }
    s->v[s->n++] = x;
}

static section *find_sec(section *secs, int ns, const char *name) {
    for (int i = 0; i < ns; i++)
        if (strcmp(secs[i].name, name) == 0) return &secs[i];
    return NULL;
}

static int need(section *secs, int ns, const char *name, int count, section **out) {
    section *s = find_sec(secs, ns, name);
    if (!s) {
        snprintf(g_err, sizeof g_err, "parameter file: missing section '%s'", name);
        return 0;
    }
    if (s->n < count) {
        snprintf(g_err, sizeof g_err, "parameter file: section '%s' has %d values, need %d",
                 name, s->n, count);
        return 0;
    }
    *out = s;
    return 1;
}

static int ival(double x) { return (int)lrint(x); }

orc_params *orc_params_load(const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) {
        snprintf(g_err, sizeof g_err, "cannot open parameter file '%s'", path);
        return NULL;
    }
    section secs[64];
    int ns = 0;
    memset(secs, 0, sizeof secs);
    section *cur = NULL;
    char line[4096];
    int in_comment = 0;
    while (fgets(line, sizeof line, f)) {
        /* strip C comments (may span lines) */
        char buf[4096];
        int k = 0;
        for (int i = 0; line[i]; i++) {
            if (in_comment) {
                if (line[i] == '*' && line[i + 1] == '/') { in_comment = 0; i++; }
                continue;
            }
            if (line[i] == '/' && line[i + 1] == '*') { in_comment = 1; i++; continue; }
            buf[k++] = line[i];
        }
        buf[k] = 0;
        char *p = buf;
        while (*p && isspace((unsigned char)*p)) p++;
        if (!*p) continue;
        if (p[0] == '#') {
            if (p[1] == '#') continue; /* "## RNAfold parameter file" banner */
            char name[64] = {0};
            sscanf(p + 1, "%63s", name);
            if (strcmp(name, "END") == 0) break;
            if (ns == 64) break;
            cur = &secs[ns++];
            strncpy(cur->name, name, sizeof cur->name - 1);
            continue;
        }
        if (!cur) continue;
        /* keep raw line for the special-loop sections */
        if (!strcmp(cur->name, "Triloops") || !strcmp(cur->name, "Tetraloops") ||
            !strcmp(cur->name, "Hexaloops")) {
            cur->lines = realloc(cur->lines, sizeof(*cur->lines) * (cur->nlines + 1));
            strncpy(cur->lines[cur->nlines], p, 63);
            cur->lines[cur->nlines][63] = 0;
            cur->nlines++;
            continue;
        }
        char *tok = strtok(p, " \t\r\n");
        while (tok) {
            if (!strcmp(tok, "INF")) sec_push(cur, ORC_INF);
            else if (!strcmp(tok, "DEF")) sec_push(cur, -50);
            else if (!strcmp(tok, "NST")) sec_push(cur, 0);
            else {
                char *end;
                double x = strtod(tok, &end);
                if (end != tok) sec_push(cur, x);
            }
            tok = strtok(NULL, " \t\r\n");
        }
    }
    fclose(f);

    orc_params *P = (orc_params *)calloc(1, sizeof(orc_params));
    section *s;
    int ok = 1;
#define NEED(name, cnt) (ok = ok && need(secs, ns, name, cnt, &s))
    if (NEED("stack", 49)) {
        for (int a = 1; a <= 7; a++)
            for (int b = 1; b <= 7; b++) P->stack[a][b] = ival(s->v[(a - 1) * 7 + (b - 1)]);
    }
    struct { const char *name; int (*t)[5][5]; } mms[] = {
        {"mismatch_hairpin", P->mmH},     {"mismatch_interior", P->mmI},
        {"mismatch_interior_1n", P->mm1nI}, {"mismatch_interior_23", P->mm23I},
        {"mismatch_multi", P->mmM},       {"mismatch_exterior", P->mmExt}};
    for (int m = 0; m < 6 && ok; m++) {
        if (NEED(mms[m].name, 175))
            for (int a = 1; a <= 7; a++)
                for (int x = 0; x < 5; x++)
                    for (int y = 0; y < 5; y++)
                        mms[m].t[a][x][y] = ival(s->v[(a - 1) * 25 + x * 5 + y]);
    }
    if (NEED("dangle5", 35))
        for (int a = 1; a <= 7; a++)
            for (int x = 0; x < 5; x++) P->d5[a][x] = ival(s->v[(a - 1) * 5 + x]);
    if (NEED("dangle3", 35))
        for (int a = 1; a <= 7; a++)
            for (int x = 0; x < 5; x++) P->d3[a][x] = ival(s->v[(a - 1) * 5 + x]);
    if (NEED("int11", 49 * 25))
        for (int a = 1; a <= 7; a++)
            for (int b = 1; b <= 7; b++)
                for (int x = 0; x < 5; x++)
                    for (int y = 0; y < 5; y++)
                        P->int11[a][b][x][y] = ival(s->v[((a - 1) * 7 + (b - 1)) * 25 + x * 5 + y]);
    if (NEED("int21", 49 * 125))
        for (int a = 1; a <= 7; a++)
            for (int b = 1; b <= 7; b++)
                for (int x = 0; x < 5; x++)
                    for (int y = 0; y < 5; y++)
                        for (int z = 0; z < 5; z++)
                            P->int21[a][b][x][y][z] =
                                ival(s->v[((a - 1) * 7 + (b - 1)) * 125 + x * 25 + y * 5 + z]);
    if (NEED("int22", 36 * 256)) {
        for (int a = 0; a < 8; a++)
            for (int b = 0; b < 8; b++)
                for (int w = 0; w < 5; w++)
                    for (int x = 0; x < 5; x++)
                        for (int y = 0; y < 5; y++)
                            for (int z = 0; z < 5; z++) P->int22[a][b][w][x][y][z] = ORC_INF;
        for (int a = 1; a <= 6; a++)
            for (int b = 1; b <= 6; b++)
                for (int w = 1; w <= 4; w++)
                    for (int x = 1; x <= 4; x++)
                        for (int y = 1; y <= 4; y++)
                            for (int z = 1; z <= 4; z++)
                                P->int22[a][b][w][x][y][z] = ival(
                                    s->v[((a - 1) * 6 + (b - 1)) * 256 + (w - 1) * 64 +
                                         (x - 1) * 16 + (y - 1) * 4 + (z - 1)]);
    }
    if (NEED("hairpin", 31)) for (int i = 0; i < 31; i++) P->hairpin[i] = ival(s->v[i]);
    if (NEED("bulge", 31)) for (int i = 0; i < 31; i++) P->bulge[i] = ival(s->v[i]);
    if (NEED("interior", 31)) for (int i = 0; i < 31; i++) P->interior[i] = ival(s->v[i]);
    if (NEED("ML_params", 6)) {
        P->MLbase = ival(s->v[0]);
        P->MLclosing = ival(s->v[2]);
        P->MLintern = ival(s->v[4]);
    }
    if (NEED("NINIO", 3)) {
        P->ninio = ival(s->v[0]);
        P->maxninio = ival(s->v[2]);
    }
    if (NEED("Misc", 5)) {
        P->DuplexInit = ival(s->v[0]);
        P->TermAU = ival(s->v[2]);
        P->lxc = s->v[4];
    }
    struct { const char *name; int len; int *n; char *seqs; int stride; int *E; int cap; } loops[] = {
        {"Triloops", 5, &P->ntri, &P->tri[0][0], 8, P->triE, 32},
        {"Tetraloops", 6, &P->ntetra, &P->tetra[0][0], 8, P->tetraE, 64},
        {"Hexaloops", 8, &P->nhexa, &P->hexa[0][0], 12, P->hexaE, 32}};
    for (int l = 0; l < 3 && ok; l++) {
        section *ls = find_sec(secs, ns, loops[l].name);
        *loops[l].n = 0;
        if (!ls) continue;
        for (int r = 0; r < ls->nlines && *loops[l].n < loops[l].cap; r++) {
            char sq[32];
            int e, h;
            if (sscanf(ls->lines[r], "%31s %d %d", sq, &e, &h) >= 2 &&
                (int)strlen(sq) == loops[l].len) {
                int idx = (*loops[l].n)++;
                strcpy(loops[l].seqs + idx * loops[l].stride, sq);
                loops[l].E[idx] = e;
            }
        }
    }
#undef NEED
    for (int i = 0; i < ns; i++) {
        free(secs[i].v);
        free(secs[i].lines);
    }
    if (!ok) {
        free(P);
        return NULL;
    }
    return P;
}

void orc_params_free(orc_params *P) { free(P); }
