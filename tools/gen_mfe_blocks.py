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
NBLK = 7           # waves 0..6 (wave 7 folds the multiloop qm / mla)
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


def partition():
    # greedy LPT over loop sizes, largest first; ties keep small u spread out
    sizes = sorted(range(MAXLOOP + 1), key=lambda u: -ucost(u))
    blocks = [[] for _ in range(NBLK)]
    load = [0] * NBLK
    for u in sizes:
        b = min(range(NBLK), key=lambda k: (load[k], len(blocks[k])))
        blocks[b].append(u)
        load[b] += ucost(u)
    return [sorted(b) for b in blocks], load


def partition_pairs():
    """14 blocks: block b and b + 7 are the two cost halves of the 7-block
    partition's block b (two lane-sets: one wave per 7-block per lane-set)."""
    global NBLK
    nb, NBLK = NBLK, 7
    blocks7, _ = partition()
    NBLK = nb
    out = [None] * 14
    for b, blk in enumerate(blocks7):
        h0, h1, c0, c1 = [], [], 0, 0
        for u in sorted(blk, key=lambda u: -ucost(u)):
            if c0 <= c1:
                h0.append(u); c0 += ucost(u)
            else:
                h1.append(u); c1 += ucost(u)
        out[b], out[b + 7] = sorted(h0), sorted(h1)
    return out, [sum(ucost(u) for u in b) for b in out]


def emit_shape_quad(u, u1):
    """Four folds per cell (uint2: free apo|holo, constrained apo|holo); every
    correction depends on the sequence only, so it is summed once (packed u32)
    and added to both words."""
    u2 = u - u1
    k = kind(u1, u2)
    L = "ldq(U.qbm, o + %d)" % u1
    if k == "gen":
        return "a.g%d = qmin(a.g%d, qadd(%s, gk[%d]));" % (u1 & 1, u1 & 1, L, min(abs(u1 - u2), KSAT))
    if k == "bul":
        return "{ const int c2 = k[%d]; a.b = qmin(a.b, qadd(%s, padd(U.ct[CT_BUL + c2], fb))); }" % (u1, L)
    if k == "1n":
        return "{ const int c2 = k[%d]; a.n = qmin(a.n, qadd(%s, padd(U.ct[CT_ONEN + c2], f1n))); }" % (u1, L)
    if k in ("stk", "b1"):
        corr = "padd(U.ct[CT_INVMM + c2], U.ct[CT_STK + C.ty8 + ((c2 * 41) >> 10)])"
        if k == "b1":
            corr = "padd(%s, U.fs1)" % corr
        return "{ const int c2 = k[%d]; a.s = qmin(a.s, qadd(%s, %s)); }" % (u1, L, corr)
    if k == "m23":
        return ("{ const int c2 = k[%d]; a.s = qmin(a.s, qadd(%s, padd(padd(U.ct[CT_INVMM + c2], U.ct[CT_M23O + c2]), C.m23f))); }"
                % (u1, L))
    tab = {"i11": "C.t11", "i12": "C.t12", "i21": "C.t21", "i22": "C.t22"}[k]
    return "a.s = qmin(a.s, qadd(%s, padd(U.ct[CT_INVMM + k[%d]], %s)));" % (L, u1, tab)


ASM_CHUNK = 16   # DP reads per inline-asm batch (VGPR budget: 2 per read)
ASM_CHUNK_CELLS = 24   # the same for the two-fold kernel (1 VGPR per read)
PIPE_CHUNK = 20        # pipelined two-fold blocks (pending table reads hold VGPRs)


TABK = ("i11", "i12", "i21", "i22")


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


def emit_group_quad_asm(u, out, cells=False, defer=False):
    """One loop size of the four-fold kernel with the group's LDS reads in
    inline-asm batches of ASM_CHUNK cells (the first also reads the inner-pair
    codes and the per-size energy record), each ending in s_waitcnt
    lgkmcnt(0): the compiler's scheduler otherwise issues these reads one at a
    time.  The loop-correction table reads that depend on the codes and all
    arithmetic stay in C++."""
    shapes = list(range(u + 1))
    spec = [u1 for u1 in shapes if kind(u1, u - u1) != "gen"]
    need_g = any(kind(u1, u - u1) == "gen" for u1 in shapes)
    ch_n = ASM_CHUNK_CELLS if cells else ASM_CHUNK
    chunks = [shapes[k:k + ch_n] for k in range(0, len(shapes), ch_n)]
    vt, ld, esz = ("uint32_t", "ds_read_b32", 4) if cells else ("uint2", "ds_read_b64", 8)
    qmin, qadd = ("pmin", "padd") if cells else ("qmin", "qadd")
    for ci_, ch in enumerate(chunks):
        outs, lines = [], []
        for u1 in ch:
            lines.append("%s %%[v%d], %%[qa] offset:%d" % (ld, u1, esz * u1))
            outs.append('[v%d] "=&v"(v%d)' % (u1, u1))
        decl = ["        %s %s;" % (vt, ", ".join("v%d" % u1 for u1 in ch))]
        if ci_ == 0:
            if spec:
                decl.append("        uint32_t %s;" % ", ".join("c%d" % u1 for u1 in spec))
            for u1 in spec:
                lines.append("ds_read_u8 %%[c%d], %%[ka] offset:%d" % (u1, u1))
                outs.append('[c%d] "=&v"(c%d)' % (u1, u1))
            krs = (["kr0"] if need_g else []) + (["kr1"] if u >= 2 else [])
            if krs:
                decl.append("        uint4 %s;" % ", ".join(krs))
            if need_g:
                lines.append("ds_read_b128 %%[kr0], %%[kk] offset:%d" % (32 * u))
                outs.append('[kr0] "=&v"(kr0)')
            if u >= 2:
                lines.append("ds_read_b128 %%[kr1], %%[kk] offset:%d" % (32 * u + 16))
                outs.append('[kr1] "=&v"(kr1)')
        lines.append("s_waitcnt lgkmcnt(0)")
        out.append("        {")
        out.extend(decl)
        out.append('        asm volatile(')
        for ln in lines:
            out.append('            "%s\\n"' % ln)
        out.append("            : " + ", ".join(outs))
        out.append('            : [qa] "v"(qa), [ka] "v"(ka), [kk] "v"(U.aku)')
        out.append('            : "memory");')
        if cells:   # constrained cells: shapes past the allowed unpaired runs take no part
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
            if k == "gen" and cells and abs(u1 - u2) >= KSAT:   # plateau: min first, add once
                pl.append(v)
            elif k == "gen":
                out.append("        a.g%d = %s(a.g%d, %s(%s, gk[%d]));" % (u1 & 1, qmin, u1 & 1, qadd, v, min(abs(u1 - u2), KSAT)))
            elif k == "bul":
                out.append("        a.b = %s(a.b, %s(%s, padd(U.ct[CT_BUL + %s], fb)));" % (qmin, qadd, v, c))
            elif k == "1n":
                out.append("        a.n = %s(a.n, %s(%s, padd(U.ct[CT_ONEN + %s], f1n)));" % (qmin, qadd, v, c))
            elif k in ("stk", "b1"):
                corr = "padd(U.ct[CT_INVMM + %s], U.ct[CT_STK + C.ty8 + ((%s * 41) >> 10)])" % (c, c)
                if k == "b1":
                    corr = "padd(%s, U.fs1)" % corr
                out.append("        a.s = %s(a.s, %s(%s, %s));" % (qmin, qadd, v, corr))
            elif k == "m23":
                out.append("        a.s = %s(a.s, %s(%s, padd(padd(U.ct[CT_INVMM + %s], U.ct[CT_M23O + %s]), C.m23f)));"
                           % (qmin, qadd, v, c, c))
            elif defer:   # the HBM table value lands later: finish at the block end
                out.append("        tv_%s = %s; ti_%s = U.ct[CT_INVMM + %s];" % (k, v, k, c))
            else:
                tab = {"i11": "C.t11", "i12": "C.t12", "i21": "C.t21", "i22": "C.t22"}[k]
                out.append("        a.s = %s(a.s, %s(%s, padd(U.ct[CT_INVMM + %s], %s)));" % (qmin, qadd, v, c, tab))
        if pl:
            out.extend(plateau_min(pl, "gk[%d]" % KSAT, "        "))
        out.append("        }")
    # declarations shared by the chunks go first
    return spec, need_g


# correction-table reads of one special shape: (tag, address kind, byte offset in ct)
CT_OFF = {"INV": 0, "BUL": 200 * 4, "ONEN": 400 * 4, "M23": 600 * 4, "STK": 800 * 4}


def spec_reads(k):
    if k == "bul":
        return [("BUL", "a")]
    if k == "1n":
        return [("ONEN", "a")]
    if k in ("stk", "b1"):
        return [("INV", "a"), ("STK", "s")]
    if k == "m23":
        return [("INV", "a"), ("M23", "a")]
    return [("INV", "a")]


def spec_expr(u, u1, R):
    """a.x = pmin(a.x, ...) of a special shape from its loaded table values R[tag]
    (the same saturating-add order as the unpipelined path)."""
    k = kind(u1, u - u1)
    V = "P%d_v%d" % (u, u1)
    if k == "bul":
        return "a.b = pmin(a.b, padd(%s, padd(%s, P%d_fb)));" % (V, R["BUL"], u)
    if k == "1n":
        return "a.n = pmin(a.n, padd(%s, padd(%s, P%d_f1n)));" % (V, R["ONEN"], u)
    if k == "stk":
        return "a.s = pmin(a.s, padd(%s, padd(%s, %s)));" % (V, R["INV"], R["STK"])
    if k == "b1":
        return "a.s = pmin(a.s, padd(%s, padd(padd(%s, %s), U.fs1)));" % (V, R["INV"], R["STK"])
    if k == "m23":
        return "a.s = pmin(a.s, padd(%s, padd(padd(%s, %s), C.m23f)));" % (V, R["INV"], R["M23"])
    tab = {"i11": "C.t11", "i12": "C.t12", "i21": "C.t21", "i22": "C.t22"}[k]
    return "a.s = pmin(a.s, padd(%s, padd(%s, %s)));" % (V, R["INV"], tab)


def pending_reads(u):
    """(asm line, output binding, input binding, result name) per table read the
    specials of group u still need; R maps (u1, tag) -> result variable."""
    lines, outs, ins, R = [], [], set(), {}
    for u1 in range(u + 1):
        k = kind(u1, u - u1)
        if k == "gen":
            continue
        for tag, ak in spec_reads(k):
            r = "R%d_%d_%s" % (u, u1, tag)
            av = "P%d_%s%d" % (u, ak, u1)
            lines.append("ds_read_b32 %%[%s], %%[%s] offset:%d" % (r, av, CT_OFF[tag]))
            outs.append('[%s] "=&v"(%s)' % (r, r))
            ins.add('[%s] "v"(%s)' % (av, av))
            R[(u1, tag)] = r
    return lines, outs, sorted(ins), R


def emit_pending_arith(u, R, out, ind):
    for u1 in range(u + 1):
        k = kind(u1, u - u1)
        if k == "gen":
            continue
        out.append(ind + spec_expr(u, u1, {tag: R[(u1, tag)] for tag, _ in spec_reads(k)}))


def emit_finish(u, out, ind):
    """The table reads + arithmetic of group u's specials on their own."""
    lines, outs, ins, R = pending_reads(u)
    out.append(ind + "{")
    out.append(ind + "    uint32_t %s;" % ", ".join(sorted(set(R.values()))))
    out.append(ind + "    asm volatile(")
    for ln in lines + ["s_waitcnt lgkmcnt(0)"]:
        out.append(ind + '        "%s\\n"' % ln)
    out.append(ind + "        : " + ", ".join(outs))
    out.append(ind + "        : " + ", ".join(ins))
    out.append(ind + '        : "memory");')
    emit_pending_arith(u, R, out, ind + "    ")
    out.append(ind + "}")


def emit_block_cells_pipe(blk, out):
    """Inline-asm path of one block with the correction-table reads of group g
    (they depend on the inner-pair codes group g's batch returns) issued in
    group g+1's batch: one LDS round trip per loop size instead of two."""
    prev = None
    for u in blk:
        spec = [u1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen"]
        need_g = len(spec) < u + 1
        if prev is None:
            out.append("    if (um < %d) return;" % u)
        else:
            out.append("    if (um < %d) {" % u)
            emit_finish(prev, out, "        ")
            out.append("        return;")
            out.append("    }")
        decl = []
        for u1 in spec:
            decl += ["P%d_v%d" % (u, u1), "P%d_a%d" % (u, u1)]
            if kind(u1, u - u1) in ("stk", "b1"):
                decl.append("P%d_s%d" % (u, u1))
        if any(kind(u1, u - u1) == "bul" for u1 in spec):
            decl.append("P%d_fb" % u)
        if any(kind(u1, u - u1) == "1n" for u1 in spec):
            decl.append("P%d_f1n" % u)
        out.append("    uint32_t %s;   // group u = %d: pending specials" % (", ".join(decl), u))
        out.append("    {   // u = %d (batched reads%s)" % (u, "" if prev is None else " + the table reads of u = %d" % prev))
        out.append("        const int o = off(dd - %d, U.N) + ci;" % (u + 2))
        out.append("        const uint32_t qa = U.aq + uint32_t(o) * 4u, ka = U.ac + uint32_t(o);")
        if need_g:
            out.append("        uint32_t gk[6];")
        shapes = list(range(u + 1))
        chunks = [shapes[k:k + PIPE_CHUNK] for k in range(0, len(shapes), PIPE_CHUNK)]
        for ci_, ch in enumerate(chunks):
            lines, outs, ins = [], [], ['[qa] "v"(qa)']
            decl = ["        uint32_t %s;" % ", ".join("v%d" % u1 for u1 in ch)]
            for u1 in ch:
                lines.append("ds_read_b32 %%[v%d], %%[qa] offset:%d" % (u1, 4 * u1))
                outs.append('[v%d] "=&v"(v%d)' % (u1, u1))
            R = {}
            if ci_ == 0:
                ins += ['[ka] "v"(ka)', '[kk] "v"(U.aku)']
                if spec:
                    decl.append("        uint32_t %s;" % ", ".join("c%d" % u1 for u1 in spec))
                for u1 in spec:
                    lines.append("ds_read_u8 %%[c%d], %%[ka] offset:%d" % (u1, u1))
                    outs.append('[c%d] "=&v"(c%d)' % (u1, u1))
                krs = (["kr0"] if need_g else []) + (["kr1"] if u >= 2 else [])
                if krs:
                    decl.append("        uint4 %s;" % ", ".join(krs))
                if need_g:
                    lines.append("ds_read_b128 %%[kr0], %%[kk] offset:%d" % (32 * u))
                    outs.append('[kr0] "=&v"(kr0)')
                if u >= 2:
                    lines.append("ds_read_b128 %%[kr1], %%[kk] offset:%d" % (32 * u + 16))
                    outs.append('[kr1] "=&v"(kr1)')
            if prev is not None and ci_ == len(chunks) - 1:   # in the smallest (last) batch
                pl, po, pi, R = pending_reads(prev)
                decl.append("        uint32_t %s;" % ", ".join(sorted(set(R.values()))))
                lines += pl
                outs += po
                ins += pi
            lines.append("s_waitcnt lgkmcnt(0)")
            out.append("        {")
            out.extend(decl)
            out.append("        asm volatile(")
            for ln in lines:
                out.append('            "%s\\n"' % ln)
            out.append("            : " + ", ".join(outs))
            out.append("            : " + ", ".join(ins))
            out.append('            : "memory");')
            if R:
                emit_pending_arith(prev, R, out, "        ")
            if ci_ == 0:
                if need_g:
                    out.append("        gk[0] = kr0.x; gk[1] = kr0.y; gk[2] = kr0.z; gk[3] = kr0.w; gk[4] = kr1.x; gk[5] = kr1.y;")
                if any(kind(u1, u - u1) == "bul" for u1 in spec):
                    out.append("        P%d_fb = kr1.z;" % u)
                if any(kind(u1, u - u1) == "1n" for u1 in spec):
                    out.append("        P%d_f1n = kr1.w;" % u)
                for u1 in spec:
                    out.append("        P%d_a%d = U.act + c%d * 4u;" % (u, u1, u1))
                    if kind(u1, u - u1) in ("stk", "b1"):
                        out.append("        P%d_s%d = U.act + uint32_t(C.ty8 + ((c%d * 41) >> 10)) * 4u;" % (u, u1, u1))
            for u1 in ch:
                u2 = u - u1
                if kind(u1, u2) == "gen":
                    out.append("        a.g%d = pmin(a.g%d, padd(v%d, gk[%d]));" % (u1 & 1, u1 & 1, u1, min(abs(u1 - u2), KSAT)))
                else:
                    out.append("        P%d_v%d = v%d;" % (u, u1, u1))
            out.append("        }")
        out.append("    }")
        out.append("    MFE_SCHED_BARRIER();   // bound the scheduling window (VGPR / SGPR pressure)")
        prev = u
    emit_finish(prev, out, "    ")


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


MERGE_SLICED = 0   # two loop sizes share a read batch while their reads fit this many VGPRs


def sliced_regs(u, S):
    spec = sum(1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen")
    ngen = u + 1 - spec
    return 2 * spec + (ngen + S - 1) // S + 4 * ((1 if ngen else 0) + (1 if u >= 2 else 0))


def sliced_parts(u, S, t):
    """One loop size of a sliced block, variable names suffixed by t: address
    lines, declarations, asm reads/outputs/inputs and the arithmetic after the
    batch."""
    spec = [u1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen"]
    gen = [u1 for u1 in range(u + 1) if kind(u1, u - u1) == "gen"]
    pre, decl, lines, outs, ins, post = [], [], [], [], [], []
    pre.append("const int o%s = off(dd - %d, U.N) + ci;" % (t, u + 2))
    pre.append("const uint32_t qa%s = U.aq + uint32_t(o%s) * 4u, ka%s = U.ac + uint32_t(o%s);" % (t, t, t, t))
    ins += ['[qa%s] "v"(qa%s)' % (t, t), '[ka%s] "v"(ka%s)' % (t, t)]
    V = lambda u1: "v%d%s" % (u1, t)
    Cc = lambda u1: "c%d%s" % (u1, t)
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
    krs = (["kr0" + t] if gen else []) + (["kr1" + t] if u >= 2 else [])
    if krs:
        decl.append("uint4 %s;" % ", ".join(krs))
    if gen:
        lines.append("ds_read_b128 %%[kr0%s], %%[kk] offset:%d" % (t, 32 * u))
        outs.append('[kr0%s] "=&v"(kr0%s)' % (t, t))
    if u >= 2:
        lines.append("ds_read_b128 %%[kr1%s], %%[kk] offset:%d" % (t, 32 * u + 16))
        outs.append('[kr1%s] "=&v"(kr1%s)' % (t, t))
    # constrained cells: shapes past the allowed unpaired runs (u1 > A or u2 > B) take no part
    post.append("if (U.mk) {")
    post.append("    const int ml = %d - C.B, mh = C.A, rr = int(C.rs >> 2);" % u)
    for u1 in spec:
        post.append("    %s = (%d >= ml && %d <= mh) ? %s : INF16;" % (V(u1), u1, u1, V(u1)))
    for k in range(nk):
        post.append("    w%d%s = (%d + rr >= ml && %d + rr <= mh) ? w%d%s : INF16;" % (k, t, gen[0] + S * k, gen[0] + S * k, k, t))
    post.append("}")
    if gen:
        post.append("const uint32_t gk%s[6] = {kr0%s.x, kr0%s.y, kr0%s.z, kr0%s.w, kr1%s.x, kr1%s.y};" % ((t,) * 7))
    if u >= 2:
        post.append("const uint32_t fb%s = kr1%s.z, f1n%s = kr1%s.w;" % (t, t, t, t))
        post.append("(void)fb%s; (void)f1n%s;" % (t, t))
    post.append("#ifndef MFE_ABL_SPEC")
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
    post.append("#endif")
    post.append("#ifndef MFE_ABL_GEN")
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
        elif S == 2:
            e = "(C.r1 ? %s : %s)" % (vals[1], vals[0])
        else:
            e = "(C.r2 ? (C.r1 ? %s : %s) : (C.r1 ? %s : %s))" % (vals[3], vals[2], vals[1], vals[0])
        post.append("a.g%d = pmin(a.g%d, padd(w%d%s, %s));" % (k & 1, k & 1, k, t, e))
    if pl:
        post.extend(x.strip() for x in plateau_min(pl, "gk%s[%d]" % (t, KSAT), "    "))
    post.append("#endif")
    return pre, decl, lines, outs, ins, post


def emit_sliced_batch(groups, S, out, ind):
    """One inline-asm read batch for the loop sizes in groups, then their arithmetic."""
    parts = [sliced_parts(u, S, t) for u, t in groups]
    out.append(ind + "{   // u = %s (%d slices)" % (", ".join(str(u) for u, _ in groups), S))
    for p in parts:
        out.extend(ind + "    " + x for x in p[0] + p[1])
    lines = sum((p[2] for p in parts), []) + ["s_waitcnt lgkmcnt(0)"]
    outs = sum((p[3] for p in parts), [])
    ins = sum((p[4] for p in parts), []) + ['[kk] "v"(U.aku)']
    out.append("#ifndef MFE_ABL_READS")
    out.append(ind + "    asm volatile(")
    for ln in lines:
        out.append(ind + '        "%s\\n"' % ln)
    out.append(ind + "        : " + ", ".join(outs))
    out.append(ind + "        : " + ", ".join(ins))
    out.append(ind + '        : "memory");')
    out.append("#else   // timing only: the batch's registers from VALU moves, no LDS")
    out.append(ind + "    asm volatile(")
    for ln in lines[:-1]:
        reg = ln.split("%[")[1].split("]")[0]
        if ln.startswith("ds_read_b128"):
            continue   # left as is (garbage energies: timing only)
        else:
            out.append(ind + '        "v_mov_b32 %%[%s], 0\\n"' % reg)
    out.append(ind + "        : " + ", ".join(outs))
    out.append(ind + "        : " + ", ".join(ins))
    out.append(ind + '        : "memory");')
    out.append("#endif")
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
    unchanged); the caller folds a.g0 / a.g1 across the slices.  Consecutive
    loop sizes share one read batch (one LDS round trip for two sizes) once the
    span admits both."""
    k = 0
    while k < len(blk):
        if k + 1 < len(blk) and sliced_regs(blk[k], S) + sliced_regs(blk[k + 1], S) <= MERGE_SLICED:
            ua, ub = blk[k], blk[k + 1]
            out.append("    if (um < %d) goto fin;" % ua)
            out.append("    if (um >= %d) {" % ub)
            emit_sliced_batch([(ua, "a"), (ub, "b")], S, out, "        ")
            out.append("    } else {")
            emit_sliced_batch([(ua, "a")], S, out, "        ")
            out.append("        goto fin;")
            out.append("    }")
            k += 2
        else:
            out.append("    if (um < %d) goto fin;" % blk[k])
            emit_sliced_batch([(blk[k], "a")], S, out, "    ")
            k += 1
    emit_table_fin(blk, out)


def gen_quad():
    blocks, load = partition_pairs()
    out = ["// GENERATED by tools/gen_mfe_blocks.py -- do not edit.",
           "// Interior-loop shapes of mfe_quad.hip (four folds per cell) in 14 blocks of LDS cost %s;" % load,
           "// blocks b and b + 7 are the halves of one 7-block (two lane-sets: wave w takes both halves).",
           "// Block b: loop sizes %s" % "; ".join("%d:%s" % (b, blk) for b, blk in enumerate(blocks)), ""]
    for b, blk in enumerate(blocks):
        out.append("__device__ __forceinline__ void mfq_blk%d(const QUni &U, const QCell &C, QAcc &a) {" % b)
        out.append("    int ci = C.i, dd = U.d, um = U.umax;")
        out.append('    asm volatile("" : "+v"(ci));')
        out.append('    asm volatile("" : "+s"(dd), "+s"(um));')
        for u in blk:
            out.append("    if (um < %d) return;" % u)
            out.append("#ifndef MFQ_NO_ASM")
            out.append("    {   // u = %d (batched reads)" % u)
            out.append("        const int o = off(dd - %d, U.N) + ci;" % (u + 2))
            out.append("        const uint32_t qa = U.aq + uint32_t(o) * 8u, ka = U.ac + uint32_t(o);")
            nspec = sum(1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen")
            out.append("        uint32_t gk[6], fb = 0, f1n = 0, cs[%d];" % max(1, nspec))
            out.append("        (void)gk; (void)fb; (void)f1n; (void)cs;")
            emit_group_quad_asm(u, out)
            out.append("    }")
            out.append("#else")
            out.append("    {   // u = %d" % u)
            out.append("        const int o = off(dd - %d, U.N) + ci;" % (u + 2))
            out.append("        const uint2 *q = U.qbm + o;")
            out.append("        const uint8_t *k = U.cc + o;")
            out.append("        (void)k;")
            need_g = any(kind(u1, u - u1) == "gen" for u1 in range(u + 1))
            if need_g:
                out.append("        const uint4 kr0 = U.ku[%d * 2];" % u)
                out.append("        const uint4 kr1 = U.ku[%d * 2 + 1];" % u)
                out.append("        const uint32_t gk[6] = {kr0.x, kr0.y, kr0.z, kr0.w, kr1.x, kr1.y};")
                out.append("        const uint32_t fb = kr1.z, f1n = kr1.w;")
            elif u >= 2:
                out.append("        const uint4 kr1 = U.ku[%d * 2 + 1];" % u)
                out.append("        const uint32_t fb = kr1.z, f1n = kr1.w;")
                out.append("        (void)f1n;")
            order = sorted(range(u + 1), key=lambda u1: kind(u1, u - u1) in ("i11", "i12", "i21", "i22"))
            for u1 in order:
                out.append("        " + emit_shape_quad(u, u1))
            nds = (u + 1) + sum(2 if kind(u1, u - u1) not in ("gen",) else 0 for u1 in range(u + 1)) + (2 if need_g else 1)
            out.append("        MFQ_GROUP_ORDER(%d);" % nds)
            out.append("    }")
            out.append("#endif")
            out.append("    MFQ_SCHED_BARRIER();")
        out.append("}")
        out.append("")
    out.append("__device__ __forceinline__ void mfq_block(int b, const QUni &U, const QCell &C, QAcc &a) {")
    out.append("    switch (b) {")
    for b in range(14):
        out.append("        case %d: mfq_blk%d(U, C, a); return;" % (b, b))
    out.append("        default: return;")
    out.append("    }")
    out.append("}")
    tb = 0
    for b, blk in enumerate(blocks):
        if any(u in (2, 3, 4) for u in blk):
            tb |= 1 << b
    out.append("")
    out.append("constexpr unsigned MFQ_TABLE_BLOCKS = 0x%xu;   // blocks with 1x1 / 1x2 / 2x1 / 2x2 shapes" % tb)
    out.append("constexpr int MFQ_NBLK = 14;")
    out.append("constexpr int MFQ_KSAT = %d;" % KSAT)
    w = max(len(b) for b in blocks) + 1
    rows = ", ".join("{" + ", ".join(str(u) for u in b + [-1] * (w - len(b))) + "}" for b in blocks)
    out.append("// loop sizes of each block, -1 terminated (runtime path for constrained cells)")
    out.append("__device__ constexpr int8_t MFQ_BLK_U[14][%d] = {%s};" % (w, rows))
    path = os.path.join(out_dir(), "mfe_quad_blocks.inc")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("quad blocks:", blocks, "load:", load, file=sys.stderr)


def emit_shape(u, u1):
    u2 = u - u1
    k = kind(u1, u2)
    L = "q[%d]" % u1
    if k == "gen":
        return "a.g%d = pmin(a.g%d, padd(%s, gk[%d]));" % (u1 & 1, u1 & 1, L, min(abs(u1 - u2), KSAT))
    if k == "bul":
        return ("{ const int c2 = k[%d]; a.b = pmin(a.b, padd(padd(%s, U.ct[CT_BUL + c2]), fb)); }"
                % (u1, L))
    if k == "1n":
        return ("{ const int c2 = k[%d]; a.n = pmin(a.n, padd(padd(%s, U.ct[CT_ONEN + c2]), f1n)); }"
                % (u1, L))
    if k in ("stk", "b1"):
        extra = "" if k == "stk" else ", U.fs1"
        body = "padd(padd(%s, U.ct[CT_INVMM + c2]), U.ct[CT_STK + C.ty8 + ((c2 * 41) >> 10)])" % L
        if extra:
            body = "padd(%s%s)" % (body, extra)
        return "{ const int c2 = k[%d]; a.s = pmin(a.s, %s); }" % (u1, body)
    if k == "m23":
        return ("{ const int c2 = k[%d]; a.s = pmin(a.s, padd(padd(padd(%s, U.ct[CT_INVMM + c2]), U.ct[CT_M23O + c2]), C.m23f)); }"
                % (u1, L))
    tab = {"i11": "C.t11", "i12": "C.t12", "i21": "C.t21", "i22": "C.t22"}[k]
    return "a.s = pmin(a.s, padd(padd(%s, U.ct[CT_INVMM + k[%d]]), %s));" % (L, u1, tab)


def main():
    blocks, load = partition()
    out = []
    out.append("// GENERATED by tools/gen_mfe_blocks.py -- do not edit.")
    out.append("// Interior-loop shapes of mfe_cells.hip in %d blocks of LDS cost %s." % (NBLK, load))
    out.append("// Block b: loop sizes %s" % "; ".join("%d:%s" % (b, blk) for b, blk in enumerate(blocks)))
    out.append("")
    for b, blk in enumerate(blocks):
        out.append("__device__ __forceinline__ void mfe_blk%d(const BUni &U, const BCell &C, Acc &a) {" % b)
        # opaque copies: keeps the per-u address arithmetic inside the block (hoisted
        # above the block switch it would stay live across all blocks)
        out.append("    int ci = C.i, dd = U.d, um = U.umax;")
        out.append('    asm volatile("" : "+v"(ci));')
        out.append('    asm volatile("" : "+s"(dd), "+s"(um));')
        out.append("#if defined(MFE_PIPE) && !defined(MFE_NO_ASM)   // table reads one group late (measured slower)")
        emit_block_cells_pipe(blk, out)
        out.append("#elif !defined(MFE_NO_ASM)")
        emit_table_decl(blk, out)
        for u in blk:
            out.append("    if (um < %d) goto fin;" % u)
            out.append("    {   // u = %d (batched reads)" % u)
            out.append("        const int o = off(dd - %d, U.N) + ci;" % (u + 2))
            out.append("        const uint32_t qa = U.aq + uint32_t(o) * 4u, ka = U.ac + uint32_t(o);")
            nspec = sum(1 for u1 in range(u + 1) if kind(u1, u - u1) != "gen")
            out.append("        uint32_t gk[6], fb = 0, f1n = 0, cs[%d];" % max(1, nspec))
            out.append("        (void)gk; (void)fb; (void)f1n; (void)cs;")
            emit_group_quad_asm(u, out, cells=True, defer=True)
            out.append("    }")
            out.append("    MFE_SCHED_BARRIER();   // bound the scheduling window (VGPR / SGPR pressure)")
        emit_table_fin(blk, out)
        out.append("#else")
        for u in blk:
            out.append("    if (um < %d) return;" % u)
            out.append("    {   // u = %d" % u)
            out.append("        const int o = off(dd - %d, U.N) + ci;" % (u + 2))
            out.append("        const uint32_t *q = U.qbm + o;")
            out.append("        const uint8_t *k = U.cc + o;")
            out.append("        (void)k;")
            # the group's energies: one LDS record per loop size (KU[u], 8 words:
            # il[u] + nin[k] for k = 0..5 (k >= 5 saturated), bulge[u], 1 x (u-1));
            # a broadcast LDS read stays in order with the data reads (a scalar load
            # would force a full lgkmcnt(0) drain at its first use)
            need_g = any(kind(u1, u - u1) == "gen" for u1 in range(u + 1))
            if need_g:
                out.append("        const uint4 kr0 = U.ku[%d * 2];" % u)
                out.append("        const uint4 kr1 = U.ku[%d * 2 + 1];" % u)
                out.append("        const uint32_t gk[6] = {kr0.x, kr0.y, kr0.z, kr0.w, kr1.x, kr1.y};")
                out.append("        const uint32_t fb = kr1.z, f1n = kr1.w;")
            elif u >= 2:
                out.append("        const uint4 kr1 = U.ku[%d * 2 + 1];" % u)
                out.append("        const uint32_t fb = kr1.z, f1n = kr1.w;")
                out.append("        (void)f1n;")
            # table shapes last (their HBM values were prefetched)
            order = sorted(range(u + 1), key=lambda u1: kind(u1, u - u1) in ("i11", "i12", "i21", "i22"))
            for n, u1 in enumerate(order):
                sp = kind(u1, u - u1) != "gen"
                if sp:
                    out.append("#ifndef MFE_ABL_SPEC")
                else:
                    out.append("#ifndef MFE_ABL_GEN")
                out.append("        " + emit_shape(u, u1))
                out.append("#endif")
                if n % SCHED_CHUNK == SCHED_CHUNK - 1 and n != len(order) - 1:
                    out.append("        __builtin_amdgcn_sched_barrier(0);")
            out.append("    }")
            out.append("    MFE_SCHED_BARRIER();   // bound the scheduling window (VGPR / SGPR pressure)")
        out.append("#endif")
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
    out.append("#ifndef MFE_NO_ASM")
    for S in (2, 4):
        for b, blk in enumerate(blocks):
            out.append("__device__ __forceinline__ void mfe_blk%d_s%d(const BUni &U, const BCell &C, Acc &a) {" % (b, S))
            out.append("    int ci = C.i, dd = U.d, um = U.umax;")
            out.append('    asm volatile("" : "+v"(ci));')
            out.append('    asm volatile("" : "+s"(dd), "+s"(um));')
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
    out.append("#endif")
    # which blocks hold the table shapes (prefetch only there)
    tb = 0
    for b, blk in enumerate(blocks):
        if any(u in (2, 3, 4) for u in blk):
            tb |= 1 << b
    out.append("constexpr unsigned MFE_TABLE_BLOCKS = 0x%xu;   // blocks with 1x1 / 1x2 / 2x1 / 2x2 shapes" % tb)
    out.append("constexpr int MFE_NBLK = %d;" % NBLK)
    out.append("constexpr int MFE_KSAT = %d;   // generic loops: nin[k] == nin[MFE_KSAT] for k >= MFE_KSAT" % KSAT)
    w = max(len(b) for b in blocks) + 1
    rows = ", ".join("{" + ", ".join(str(u) for u in b + [-1] * (w - len(b))) + "}" for b in blocks)
    out.append("// loop sizes of each block, -1 terminated (runtime path for constrained cells)")
    out.append("__device__ constexpr int8_t MFE_BLK_U[%d][%d] = {%s};" % (NBLK, w, rows))
    path = os.path.join(out_dir(), "mfe_blocks.inc")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("blocks:", blocks, "load:", load, file=sys.stderr)


if __name__ == "__main__":
    main()
    gen_quad()
