#!/usr/bin/env python3
"""Generate addapt_amd/csrc/mfe_blocks.inc: the interior-loop shapes of the
lanes = cells MFE kernel (mfe_cells.hip) as straight-line code.

A closing pair (i, j) reaches an inner pair (p, q) = (i+1+u1, j-1-u2) through a
loop of size u = u1 + u2 <= 30 (ViennaRNA MAXLOOP; E_IntLoop cases restated in
oracle/fold.c E_int).  For one anti-diagonal every lane holds one cell, so a
shape (u, u1) is ONE LDS read per lane at a per-lane base for u and the
immediate offset 4*u1, plus a packed 16-bit add and min.  The 496 shapes are cut
into 8 blocks of about equal LDS cost; each block holds whole loop sizes u
(one base per u) spread over the u range, so every block has work at small
spans too.  Within a block the sizes ascend and the block returns at the first
u above the span's umax.

Shape kinds (accumulator):
  stack (0,0), bulge 1 (0,1)/(1,0)          -> a.s  (stack table via the inner code)
  1x1, 1x2, 2x1, 2x2                         -> a.s  (prefetched HBM table value)
  2x3 / 3x2                                  -> a.s  (+ outer mismatch23 per lane)
  bulge u >= 2 (0,u)/(u,0)                   -> a.b  (+ TermAU of the outer pair later)
  1 x n (1,n)/(n,1), n >= 3                  -> a.n  (+ outer mismatch1n later)
  generic u1, u2 >= 2, u >= 6                -> a.g  (+ outer mismatchI later)
"""
import os
import sys

def out_dir():
    """addapt_amd/csrc, or ADX_GEN_OUT (tests regenerate into a scratch directory)."""
    return os.environ.get("ADX_GEN_OUT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "addapt_amd", "csrc")


MAXLOOP = 30
# PAIR: the blocks of the two-diagonals-per-barrier kernel (mfe_pair.hip) --
# loop sizes u >= 2 only (the stack and bulge-1 shapes run in its finalize), and
# a lane-set holds cells of two diagonals d, d+1: a lane's inner cells sit at
# off(d - 2 - u) + ci + hb * u, with ci = i + hb * (N - d + 2) and hb = 1 on the
# lanes of diagonal d + 1 (per-lane, set once per lane-set)
PAIR = False
NBLK = int(os.environ.get("ADX_GEN_NBLK", "7"))   # block waves 0..NBLK-1 (wave 7 folds the multiloop qm / mla)
SCHED_CHUNK = 1000 # shapes per scheduling window (whole loop sizes)
KSAT = 5           # nin[k] == nin[KSAT] for k >= KSAT (checked on the host)


def kind(u1, u2):
    nl, ns = max(u1, u2), min(u1, u2)
    if nl == 0:
        return "stk"
    if ns == 0:
        return "b1" if nl == 1 else "bul"
    if ns == 1:
        if nl == 1:
            return "i11"
        if nl == 2:
            return "i12" if u1 == 1 else "i21"
        return "1n"
    if ns == 2 and nl == 2:
        return "i22"
    if ns == 2 and nl == 3:
        return "m23"
    return "gen"


# LDS reads per shape kind (qbm + code + table reads)
COST = {"stk": 4, "b1": 4, "bul": 3, "1n": 3, "i11": 3, "i12": 3, "i21": 3, "i22": 3, "m23": 4, "gen": 1}


def ucost(u):
    return sum(COST[kind(u1, u - u1)] for u1 in range(u + 1))


def edges(u):
    """The four edge shapes of a loop size u >= 4 -- bulges (0,u) (u,0), 1 x n
    loops (1,u-1) (u-1,1) -- spread over the lane slices of a sliced block."""
    return [0, u, 1, u - 1] if u >= 4 else []


def scost(u, S):
    """LDS cost per lane of loop size u in a block with S lanes per cell: the
    edge shapes spread over the slices, other special shapes in every slice,
    generic shapes 1/S each."""
    if S == 1:
        return ucost(u)
    e = edges(u)
    spec = [u1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen" and u1 not in e]
    ngen = sum(1 for u1 in range(u + 1) if kind(u1, u - u1) == "gen")
    return (len(e) // S) * 3 + sum(COST[kind(u1, u - u1)] for u1 in spec) + (ngen + S - 1) // S


# one-wave roles riding on block waves (mfe_cells.hip), in block-cost units,
# from the stamps (tools/mfe_mc_stamps.py): finalize lane-set 0 on wave 1, the
# qm1 column minima on wave 3, the list + records on wave 4 (q5 runs on the qm
# wave 7, which has slack: 1.248M -> 1.266M MC steps/s; finalize on wave 1
# instead of 6: +0.7-0.9 %; profiles/r04y_ab_roles.txt, r04z_ab_roles.txt)
ROLES4 = "1:8,3:5,4:10" if NBLK == 7 else ""   # NBLK <= 4: the roles have waves of their own
# pair kernel (mfe_pair.hip; cycles from tools/mfe_pair_stamps.py at ~4k per
# unit): the split parts of span d on wave 0 and of d+1 on wave 2, q5 of two
# columns on wave 3, the lists on wave 1 (round 5; wave 4 before), the finalize's second lane-set
# (spans < 38) on wave 6; its first lane-set has wave 7 to itself
PAIR_ROLES4 = "0:22,1:22,2:22,3:16,6:5"


def umin():
    return 2 if PAIR else 0


def role_loads(S):
    """Per-wave cost of the roles (ADX_GEN_ROLES4 overrides, "wave:cost,...").
    Only the 4-lanes-per-cell partition uses them: it serves ~96 % of an MC
    refold's diagonals, the other two keep equal block costs."""
    init = [0] * NBLK
    env = "ADX_GEN_PAIR_ROLES4" if PAIR else "ADX_GEN_ROLES4"
    spec = os.environ.get(env, PAIR_ROLES4 if PAIR else ROLES4) if S == 4 else ""
    for item in filter(None, spec.split(",")):
        w, c = item.split(":")
        init[int(w)] = int(c)
    return init


def partition(S=1):
    # greedy LPT over loop sizes, largest first; ties keep small u spread out
    sizes = sorted(range(umin(), MAXLOOP + 1), key=lambda u: (-scost(u, S), -ucost(u)))
    blocks = [[] for _ in range(NBLK)]
    load = role_loads(S)
    for u in sizes:
        b = min(range(NBLK), key=lambda k: (load[k], len(blocks[k])))
        blocks[b].append(u)
        load[b] += scost(u, S)
    return [sorted(b) for b in blocks], load


ASM_CHUNK = 24   # DP reads per inline-asm batch (1 VGPR per read)
# sliced modes whose blocks get a batched path for spans that reach every loop
# size of the block (umax >= its largest u): the sizes' reads in batches of at
# most FULL_READS per lane, one LDS round trip each instead of one per size
# (4 lanes per cell: 1.013M -> 1.054M MC steps/s; larger batches spill, and
# the 2-lanes path spills 40 VGPRs with it)
FULL_READS = int(os.environ.get("ADX_GEN_FULL_READS", "24"))
FULL_BATCH = tuple(int(x) for x in os.environ.get("ADX_GEN_FULL", "4").split(",") if x)


TABK = ("i11", "i12", "i21", "i22")

# 4 lanes per cell: generic shapes whose energies differ between the slices of a
# read row k (|2 u1 - u| < KSAT for some slice) take them from a per-lane LDS
# table (mfe_cells.hip CL::e4, slot q at byte 16 q + 4 r for slice r) read in the
# batch, instead of a per-lane select among the record's scalar values
ETAB4 = os.environ.get("ADX_GEN_ETAB4", "1") == "1"


def gen_rows(u, S):
    """Per read row k of loop size u with S slices: the asymmetry index
    min(|2 u1 - u|, KSAT) of each slice (None past the generic shapes)."""
    gen = [u1 for u1 in range(u + 1) if kind(u1, u - u1) == "gen"]
    if not gen:
        return []
    nk = (len(gen) + S - 1) // S
    return [[min(abs(2 * u1 - u), KSAT) if u1 in gen else None
             for u1 in (gen[0] + r + S * k for r in range(S))] for k in range(nk)]


def e4_slots():
    """(u, k, asym per slice) of every 4-slice row with differing energies."""
    out = []
    for u in range(MAXLOOP + 1):
        for k, row in enumerate(gen_rows(u, 4)):
            if len(set(row)) > 1:
                out.append((u, k, row))
    return out


E4_SLOT = {(u, k): q for q, (u, k, _) in enumerate(e4_slots())}


def plateau_min(vals, e, ind):
    """Generic shapes with the saturated (plateau) energy e: a pairwise min tree,
    then one add (no saturation for possible values, and stored impossible
    values stay impossible: the same result as adding first)."""
    vals = list(vals)
    lines = []
    n = 0
    while len(vals) > 1:
        nxt = []
        for a in range(0, len(vals) - 1, 2):
            t = "pm%d" % n
            n += 1
            lines.append(ind + "const u32 %s = pmin(%s, %s);" % (t, vals[a], vals[a + 1]))
            nxt.append(t)
        if len(vals) % 2:
            nxt.append(vals[-1])
        vals = nxt
    lines.append(ind + "a.g0 = pmin(a.g0, padd(%s, %s));" % (vals[0], e))
    return ["        {"] + lines + ["        }"] if False else [ind[:-4] + "{"] + lines + [ind[:-4] + "}"]


def emit_group_asm(u, out):
    """One loop size with the group's LDS reads in inline-asm batches of
    ASM_CHUNK cells (the first also reads the inner-pair codes and the per-size
    energy record), each ending in s_waitcnt lgkmcnt(0): the compiler's
    scheduler otherwise issues these reads one at a time.  The loop-correction
    table reads that depend on the codes and all arithmetic stay in C++; the
    1x1 .. 2x2 shapes wait for their HBM table values until the block end."""
    shapes = list(range(u + 1))
    spec = [u1 for u1 in shapes if kind(u1, u - u1) != "gen"]
    need_g = any(kind(u1, u - u1) == "gen" for u1 in shapes)
    chunks = [shapes[k:k + ASM_CHUNK] for k in range(0, len(shapes), ASM_CHUNK)]
    for ci_, ch in enumerate(chunks):
        outs, lines = [], []
        for u1 in ch:
            lines.append("ds_read_b32 %%[v%d], %%[qa] offset:%d" % (u1, 4 * u1))
            outs.append('[v%d] "=&v"(v%d)' % (u1, u1))
        decl = ["        uint32_t %s;" % ", ".join("v%d" % u1 for u1 in ch)]
        if ci_ == 0:
            if spec:
                decl.append("        uint32_t %s;" % ", ".join("c%d" % u1 for u1 in spec))
            for u1 in spec:
                lines.append("ds_read_u8 %%[c%d], %%[ka] offset:%d" % (u1, u1))
                outs.append('[c%d] "=&v"(c%d)' % (u1, u1))
            # the loop size's energy record: uniform, scalar loads (DevScaled::ku16)
            if need_g:
                decl.append("        const uint4 kr0 = kload(kg, %d);" % (2 * u))
            if u >= 2:
                decl.append("        const uint4 kr1 = kload(kg, %d);" % (2 * u + 1))
        lines.append("s_waitcnt lgkmcnt(0)")
        out.append("        {")
        out.extend(decl)
        out.append('        asm volatile(')
        for ln in lines:
            out.append('            "%s\\n"' % ln)
        out.append("            : " + ", ".join(outs))
        out.append('            : [qa] "v"(qa), [ka] "v"(ka)')
        out.append('            : "memory");')
        # constrained cells: shapes past the allowed unpaired runs take no part
        out.append("        if (U.mk) {")
        out.append("            const int ml = %d - C.B, mh = C.A;" % u)
        for u1 in ch:
            out.append("            v%d = (%d >= ml && %d <= mh) ? v%d : INF16;" % (u1, u1, u1, u1))
        out.append("        }")
        if ci_ == 0:
            if need_g:
                out.append("        gk[0] = kr0.x; gk[1] = kr0.y; gk[2] = kr0.z; gk[3] = kr0.w; gk[4] = kr1.x; gk[5] = kr1.y;")
            if u >= 2:
                out.append("        fb = kr1.z; f1n = kr1.w;")
            for u1 in spec:
                out.append("        cs[%d] = c%d;" % (spec.index(u1), u1))
        pl = []
        for u1 in ch:
            u2 = u - u1
            k = kind(u1, u2)
            v = "v%d" % u1
            c = "cs[%d]" % spec.index(u1) if u1 in spec else None
            if k == "gen" and abs(u1 - u2) >= KSAT:   # plateau: min first, add once
                pl.append(v)
            elif k == "gen":
                out.append("        a.g%d = pmin(a.g%d, padd(%s, gk[%d]));" % (u1 & 1, u1 & 1, v, min(abs(u1 - u2), KSAT)))
            elif k == "bul":
                out.append("        a.b = pmin(a.b, padd(%s, padd(U.ct[CT_BUL + %s], fb)));" % (v, c))
            elif k == "1n":
                out.append("        a.n = pmin(a.n, padd(%s, padd(U.ct[CT_ONEN + %s], f1n)));" % (v, c))
            elif k in ("stk", "b1"):
                corr = "padd(U.ct[CT_INVMM + %s], U.ct[CT_STK + C.ty8 + ((%s * 41) >> 10)])" % (c, c)
                if k == "b1":
                    corr = "padd(%s, U.fs1)" % corr
                out.append("        a.s = pmin(a.s, padd(%s, %s));" % (v, corr))
            elif k == "m23":
                out.append("        a.s = pmin(a.s, padd(%s, padd(padd(U.ct[CT_INVMM + %s], U.ct[CT_M23O + %s]), C.m23f)));"
                           % (v, c, c))
            else:   # the HBM table value lands later: finish at the block end
                out.append("        tv_%s = %s; ti_%s = U.ct[CT_INVMM + %s];" % (k, v, k, c))
        if pl:
            out.extend(plateau_min(pl, "gk[%d]" % KSAT, "        "))
        out.append("        }")


def table_kinds(blk):
    return sorted({kind(u1, u - u1) for u in blk for u1 in range(u + 1)} & set(TABK))


def emit_table_decl(blk, out):
    """1x1 .. 2x2 shapes wait for their HBM table values until the block end."""
    for k in table_kinds(blk):
        out.append("    u32 tv_%s = INF16, ti_%s = 0u;" % (k, k))


def emit_table_fin(blk, out):
    out.append("fin:")
    for k in table_kinds(blk):
        tab = {"i11": "C.t11", "i12": "C.t12", "i21": "C.t21", "i22": "C.t22"}[k]
        out.append("    a.s = pmin(a.s, padd(tv_%s, padd(ti_%s, %s)));" % (k, k, tab))
    out.append("    return;")


def sliced_parts(u, S, t):
    """One loop size of a sliced block, variable names suffixed by t: address
    lines, declarations, asm reads/outputs/inputs and the arithmetic after the
    batch.  Loop sizes u >= 4 spread their edge shapes over the slices: with
    S = 4 slice r reads edge n1 = C.ea + C.eb * u (bulges on slices 0, 1, 1 x n
    on 2, 3: accumulator a.e, the outer term per slice is added by the caller),
    with S = 2 slice r reads the bulge n1 = C.eb * u and the 1 x n loop
    n1 = C.ea + C.eb * u."""
    ed = edges(u)
    spec = [u1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen" and u1 not in ed]
    gen = [u1 for u1 in range(u + 1) if kind(u1, u - u1) == "gen"]
    pre, decl, lines, outs, ins, post = [], [], [], [], [], []
    pre.append("const int o%s = off(dd - %d, U.N) + ci%s;" % (t, u + 2, (" + hb * %d" % u) if PAIR else ""))
    pre.append("const uint32_t qa%s = U.aq + uint32_t(o%s) * 4u, ka%s = U.ac + uint32_t(o%s);" % (t, t, t, t))
    ins += ['[qa%s] "v"(qa%s)' % (t, t), '[ka%s] "v"(ka%s)' % (t, t)]
    V = lambda u1: "v%d%s" % (u1, t)
    Cc = lambda u1: "c%d%s" % (u1, t)
    # edge reads: (name, per-lane n1 expression, kind)
    eds = []
    if ed and S == 4:
        eds = [("e", "ea + eb * %d" % u, "edge")]
    elif ed and S == 2:
        eds = [("b", "eb * %d" % u, "bul"), ("n", "ea + eb * %d" % u, "1n")]
    for nm, ex, _ in eds:
        pre.append("const int n%s%s = %s;" % (nm, t, ex))
        pre.append("const uint32_t q%s%s = qa%s + uint32_t(n%s%s) * 4u, k%s%s = ka%s + uint32_t(n%s%s);"
                   % (nm, t, t, nm, t, nm, t, t, nm, t))
        ins += ['[q%s%s] "v"(q%s%s)' % (nm, t, nm, t), '[k%s%s] "v"(k%s%s)' % (nm, t, nm, t)]
        decl.append("uint32_t v%s%s, c%s%s;" % (nm, t, nm, t))
        lines.append("ds_read_b32 %%[v%s%s], %%[q%s%s]" % (nm, t, nm, t))
        outs.append('[v%s%s] "=&v"(v%s%s)' % (nm, t, nm, t))
        lines.append("ds_read_u8 %%[c%s%s], %%[k%s%s]" % (nm, t, nm, t))
        outs.append('[c%s%s] "=&v"(c%s%s)' % (nm, t, nm, t))
    if spec:
        decl.append("uint32_t %s;" % ", ".join(V(u1) for u1 in spec))
        decl.append("uint32_t %s;" % ", ".join(Cc(u1) for u1 in spec))
    for u1 in spec:
        lines.append("ds_read_b32 %%[%s], %%[qa%s] offset:%d" % (V(u1), t, 4 * u1))
        outs.append('[%s] "=&v"(%s)' % (V(u1), V(u1)))
    for u1 in spec:
        lines.append("ds_read_u8 %%[%s], %%[ka%s] offset:%d" % (Cc(u1), t, u1))
        outs.append('[%s] "=&v"(%s)' % (Cc(u1), Cc(u1)))
    nk = 0
    if gen:
        g0 = gen[0]
        nk = (len(gen) + S - 1) // S
        pre.append("const uint32_t qg%s = qa%s + C.rs + %du;   // this slice's first generic shape" % (t, t, 4 * g0))
        ins.append('[qg%s] "v"(qg%s)' % (t, t))
        decl.append("uint32_t %s;" % ", ".join("w%d%s" % (k, t) for k in range(nk)))
        for k in range(nk):
            lines.append("ds_read_b32 %%[w%d%s], %%[qg%s] offset:%d" % (k, t, t, 4 * S * k))
            outs.append('[w%d%s] "=&v"(w%d%s)' % (k, t, k, t))
    etab = []   # rows k whose energies come from the per-lane table
    if ETAB4 and S == 4:
        for k in range(nk):
            if (u, k) in E4_SLOT:
                etab.append(k)
                decl.append("uint32_t e%d%s;" % (k, t))
                lines.append("ds_read_b32 %%[e%d%s], %%[qt%s] offset:%d" % (k, t, t, 16 * E4_SLOT[(u, k)]))
                outs.append('[e%d%s] "=&v"(e%d%s)' % (k, t, k, t))
        if etab:
            ins.append('[qt%s] "v"(C.ee)' % t)
    # the loop size's energy record: uniform, scalar loads (DevScaled::ku16)
    if gen:
        decl.append("const uint4 kr0%s = kload(kg, %d);" % (t, 2 * u))
    if u >= 2:
        decl.append("const uint4 kr1%s = kload(kg, %d);" % (t, 2 * u + 1))
    # constrained cells: shapes past the allowed unpaired runs (u1 > A or u2 > B) take no part
    post.append("if (U.mk) {")
    post.append("    const int ml = %d - C.B, mh = C.A, rr = int(C.rs >> 2);" % u)
    for u1 in spec:
        post.append("    %s = (%d >= ml && %d <= mh) ? %s : INF16;" % (V(u1), u1, u1, V(u1)))
    for nm, _, _ in eds:
        post.append("    v%s%s = (n%s%s >= ml && n%s%s <= mh) ? v%s%s : INF16;" % ((nm, t) * 4))
    if PAIR and nk:   # the slice offset folded into the bounds once (no per-position lane constants)
        post.append("    const int gl = ml - rr, gh = mh - rr;")
    for k in range(nk):
        if PAIR:
            post.append("    w%d%s = (%d >= gl && %d <= gh) ? w%d%s : INF16;" % (k, t, gen[0] + S * k, gen[0] + S * k, k, t))
        else:
            post.append("    w%d%s = (%d + rr >= ml && %d + rr <= mh) ? w%d%s : INF16;" % (k, t, gen[0] + S * k, gen[0] + S * k, k, t))
    post.append("}")
    if gen:
        post.append("const uint32_t gk%s[6] = {kr0%s.x, kr0%s.y, kr0%s.z, kr0%s.w, kr1%s.x, kr1%s.y};" % ((t,) * 7))
    if u >= 2:
        post.append("const uint32_t fb%s = kr1%s.z, f1n%s = kr1%s.w;" % (t, t, t, t))
        post.append("(void)fb%s; (void)f1n%s;" % (t, t))
    for nm, _, k in eds:
        v, c = "v%s%s" % (nm, t), "c%s%s" % (nm, t)
        if k == "edge":
            post.append("a.e = pmin(a.e, padd(%s, padd(U.ct[C.ctb + %s], C.r2 ? f1n%s : fb%s)));" % (v, c, t, t))
        elif k == "bul":
            post.append("a.b = pmin(a.b, padd(%s, padd(U.ct[CT_BUL + %s], fb%s)));" % (v, c, t))
        else:
            post.append("a.n = pmin(a.n, padd(%s, padd(U.ct[CT_ONEN + %s], f1n%s)));" % (v, c, t))
    for u1 in spec:
        k = kind(u1, u - u1)
        v, c = V(u1), Cc(u1)
        if k == "bul":
            post.append("a.b = pmin(a.b, padd(%s, padd(U.ct[CT_BUL + %s], fb%s)));" % (v, c, t))
        elif k == "1n":
            post.append("a.n = pmin(a.n, padd(%s, padd(U.ct[CT_ONEN + %s], f1n%s)));" % (v, c, t))
        elif k in ("stk", "b1"):
            corr = "padd(U.ct[CT_INVMM + %s], U.ct[CT_STK + C.ty8 + ((%s * 41) >> 10)])" % (c, c)
            if k == "b1":
                corr = "padd(%s, U.fs1)" % corr
            post.append("a.s = pmin(a.s, padd(%s, %s));" % (v, corr))
        elif k == "m23":
            post.append("a.s = pmin(a.s, padd(%s, padd(padd(U.ct[CT_INVMM + %s], U.ct[CT_M23O + %s]), C.m23f)));" % (v, c, c))
        else:
            post.append("tv_%s = %s; ti_%s = U.ct[CT_INVMM + %s];" % (k, v, k, c))
    pl = []
    for k in range(nk):
        vals = []
        for r in range(S):
            u1 = gen[0] + r + S * k
            vals.append("gk%s[%d]" % (t, min(abs(2 * u1 - u), KSAT)) if u1 in gen else "INF16")
        if len(set(vals)) == 1 and vals[0] == "gk%s[%d]" % (t, KSAT):
            pl.append("w%d%s" % (k, t))
            continue
        if len(set(vals)) == 1:
            e = vals[0]
        elif k in etab:
            e = "e%d%s" % (k, t)
        elif S == 2:
            e = "(C.r1 ? %s : %s)" % (vals[1], vals[0])
        else:
            e = "(C.r2 ? (C.r1 ? %s : %s) : (C.r1 ? %s : %s))" % (vals[3], vals[2], vals[1], vals[0])
        post.append("a.g%d = pmin(a.g%d, padd(w%d%s, %s));" % (k & 1, k & 1, k, t, e))
    if pl:
        post.extend(x.strip() for x in plateau_min(pl, "gk%s[%d]" % (t, KSAT), "    "))
    # only the address operands the batch's reads use (an unused input still holds a VGPR)
    ins = [x for x in ins if "%%[%s]" % x.split("]")[0][1:] in "".join(lines)]
    return pre, decl, lines, outs, ins, post


def emit_sliced_batch(groups, S, out, ind):
    """One inline-asm read batch for the loop sizes in groups, then their arithmetic."""
    parts = [sliced_parts(u, S, t) for u, t in groups]
    out.append(ind + "{   // u = %s (%d slices)" % (", ".join(str(u) for u, _ in groups), S))
    for p in parts:
        out.extend(ind + "    " + x for x in p[0] + p[1])
    lines = sum((p[2] for p in parts), []) + ["s_waitcnt lgkmcnt(0)"]
    outs = sum((p[3] for p in parts), [])
    ins = sum((p[4] for p in parts), [])
    out.append(ind + "    asm volatile(")
    for ln in lines:
        out.append(ind + '        "%s\\n"' % ln)
    out.append(ind + "        : " + ", ".join(outs))
    out.append(ind + "        : " + ", ".join(ins))
    out.append(ind + '        : "memory");')
    for p in parts:
        out.extend(ind + "    " + x for x in p[5])
    out.append(ind + "}")
    out.append(ind + "MFE_SCHED_BARRIER();")


def emit_block_cells_sliced(blk, S, out):
    """Inline-asm path of one block with S lanes per cell (S = 2, 4): lane slice
    r = 0..S-1 reads the generic shapes u1 = 2 + r + S*k of each loop size (one
    per-lane base + immediate offsets), so a diagonal with <= 64/S pairable cells
    runs the generic shapes in 1/S of the instructions.  Every slice also runs
    the special shapes (counting a shape in several slices leaves the minimum
    unchanged); the caller folds a.g0 / a.g1 across the slices."""
    if S in FULL_BATCH:
        # every loop size of the block fits the span: the whole block's reads in
        # one batch (one LDS round trip, then one for the dependent code reads)
        out.append("    if (um >= %d) {" % max(blk))
        groups, cur, nrd = [], [], 0
        for u in blk:   # batches of at most FULL_READS reads per lane
            r = len(sliced_parts(u, S, "x")[2])
            if cur and nrd + r > FULL_READS:
                groups.append(cur)
                cur, nrd = [], 0
            cur.append((u, "u%d" % u))
            nrd += r
        groups.append(cur)
        for g in groups:
            emit_sliced_batch(g, S, out, "        ")
        out.append("        goto fin;")
        out.append("    }")
    for u in blk:
        out.append("    if (um < %d) goto fin;" % u)
        emit_sliced_batch([(u, "a")], S, out, "    ")
    emit_table_fin(blk, out)


# the pair kernel's block waves (ADX_GEN_PAIR_NBLK; its output file name
# ADX_GEN_PAIR_OUT, for A/B builds of another wave count)
PAIR_NBLK = int(os.environ.get("ADX_GEN_PAIR_NBLK", str(NBLK)))


def main():
    global PAIR, NBLK
    cells_nblk = NBLK
    only = os.environ.get("ADX_GEN_ONLY")   # "pair" / "cells": one file
    for PAIR in (False, True):
        if only and only != ("pair" if PAIR else "cells"):
            continue
        NBLK = PAIR_NBLK if PAIR else cells_nblk
        emit_file()


def emit_file():
    blocks, load = partition()
    out = []
    out.append("// GENERATED by tools/gen_mfe_blocks.py -- do not edit.")
    if PAIR:
        out.append("// Pair variant (mfe_pair.hip): loop sizes u >= 2, per-lane diagonal offset hb.")
    out.append("// Interior-loop shapes of mfe_cells.hip in %d blocks of LDS cost %s." % (NBLK, load))
    out.append("// Block b: loop sizes %s" % "; ".join("%d:%s" % (b, blk) for b, blk in enumerate(blocks)))
    out.append("")
    for b, blk in enumerate(blocks):
        out.append("__device__ __forceinline__ void mfe_blk%d(const BUni &U, const BCell &C, Acc &a) {" % b)
        # opaque copies: keeps the per-u address arithmetic inside the block (hoisted
        # above the block switch it would stay live across all blocks)
        out.append("    int ci = C.i, dd = U.d, um = U.umax;")
        out.append('    asm volatile("" : "+v"(ci));')
        if PAIR:
            out.append('    int hb = C.hb;')
            out.append('    asm volatile("" : "+v"(hb));')
        out.append('    asm volatile("" : "+s"(dd), "+s"(um));')
        out.append('    const kc_u32 *kg = kconst(U.kg);   // opaque: the record loads stay at their use (s_load, SGPRs)')
        out.append('    asm volatile("" : "+s"(kg));')
        emit_table_decl(blk, out)
        for u in blk:
            out.append("    if (um < %d) goto fin;" % u)
            out.append("    {   // u = %d (batched reads)" % u)
            out.append("        const int o = off(dd - %d, U.N) + ci%s;" % (u + 2, (" + hb * %d" % u) if PAIR else ""))
            out.append("        const uint32_t qa = U.aq + uint32_t(o) * 4u, ka = U.ac + uint32_t(o);")
            nspec = sum(1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen")
            out.append("        uint32_t gk[6], fb = 0, f1n = 0, cs[%d];" % max(1, nspec))
            out.append("        (void)gk; (void)fb; (void)f1n; (void)cs;")
            emit_group_asm(u, out)
            out.append("    }")
            out.append("    MFE_SCHED_BARRIER();   // bound the scheduling window (VGPR / SGPR pressure)")
        emit_table_fin(blk, out)
        out.append("}")
        out.append("")
    out.append("__device__ __forceinline__ void mfe_block(int b, const BUni &U, const BCell &C, Acc &a) {")
    out.append("    switch (b) {")
    for b in range(NBLK):
        out.append("        case %d: mfe_blk%d(U, C, a); return;" % (b, b))
    out.append("        default: return;")
    out.append("    }")
    out.append("}")
    out.append("")
    for S in (2, 4):
        sblocks, sload = partition(S)
        out.append("// %d lanes per cell: blocks of LDS cost %s: %s" % (S, sload, "; ".join("%d:%s" % (b, blk) for b, blk in enumerate(sblocks))))
        for b, blk in enumerate(sblocks):
            out.append("__device__ __forceinline__ void mfe_blk%d_s%d(const BUni &U, const BCell &C, Acc &a) {" % (b, S))
            out.append("    int ci = C.i, dd = U.d, um = U.umax, ea = C.ea, eb = C.eb;")
            out.append('    asm volatile("" : "+v"(ci), "+v"(ea), "+v"(eb));')
            if PAIR:
                out.append('    int hb = C.hb;')
                out.append('    asm volatile("" : "+v"(hb));')
            out.append('    asm volatile("" : "+s"(dd), "+s"(um));')
            out.append('    const kc_u32 *kg = kconst(U.kg);   // opaque: the record loads stay at their use (s_load, SGPRs)')
            out.append('    asm volatile("" : "+s"(kg));')
            emit_table_decl(blk, out)
            emit_block_cells_sliced(blk, S, out)
            out.append("}")
            out.append("")
        out.append("__device__ __forceinline__ void mfe_block_s%d(int b, const BUni &U, const BCell &C, Acc &a) {" % S)
        out.append("    switch (b) {")
        for b in range(NBLK):
            out.append("        case %d: mfe_blk%d_s%d(U, C, a); return;" % (b, b, S))
        out.append("        default: return;")
        out.append("    }")
        out.append("}")
        out.append("")
    # which blocks hold the table shapes (prefetch only there), per lanes per cell
    for S in (1, 2, 4):
        tb = 0
        for b, blk in enumerate(partition(S)[0]):
            if any(u in (2, 3, 4) for u in blk):
                tb |= 1 << b
        out.append("constexpr unsigned MFE_TABLE_BLOCKS%s = 0x%xu;   // blocks with 1x1 / 1x2 / 2x1 / 2x2 shapes%s"
                   % ("" if S == 1 else "_S%d" % S, tb, "" if S == 1 else " (%d lanes per cell)" % S))
    # the block (wave) of every loop size per lanes-per-cell mode (1, 2, 4): the
    # kernels load a table energy / factor only on the wave whose block reads it
    rows = []
    for S in (1, 2, 4):
        wb = [-1] * (MAXLOOP + 1)
        for b, blk in enumerate(partition(S)[0]):
            for u in blk:
                wb[u] = b
        rows.append("{%s}" % ", ".join(str(x) for x in wb))
    out.append("constexpr signed char MFE_SIZE_BLOCK[3][%d] = {%s};   // [log2 lanes per cell][u] -> block"
               % (MAXLOOP + 1, ", ".join(rows)))
    sl = e4_slots() if ETAB4 else []
    out.append("// per-lane generic energies of the 4-lanes-per-cell blocks: slot q holds loop size")
    out.append("// MFE_E4_U[q] and, for slice r, the Ninio index MFE_E4_A[q][r] (-1: no shape)")
    out.append("constexpr int MFE_E4_SLOTS = %d;" % len(sl))
    out.append("constexpr signed char MFE_E4_U[%d] = {%s};" % (max(1, len(sl)), ", ".join(str(u) for u, _, _ in sl) or "0"))
    out.append("constexpr signed char MFE_E4_A[%d][4] = {%s};" % (max(1, len(sl)), ", ".join(
        "{%s}" % ", ".join(str(-1 if a is None else a) for a in row) for _, _, row in sl) or "{-1, -1, -1, -1}"))
    out.append("constexpr int MFE_NBLK = %d;" % NBLK)
    out.append("constexpr int MFE_KSAT = %d;   // generic loops: nin[k] == nin[MFE_KSAT] for k >= MFE_KSAT" % KSAT)
    path = os.path.join(out_dir(), os.environ.get("ADX_GEN_PAIR_OUT", "mfe_pair_blocks.inc") if PAIR
                        else "mfe_blocks.inc")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("blocks:", blocks, "load:", load, file=sys.stderr)


if __name__ == "__main__":
    main()
