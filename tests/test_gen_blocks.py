"""Host checks of the interior-loop shape generator (tools/gen_mfe_blocks.py)
behind mfe_cells.hip: every loop size in exactly one block,
the sliced blocks' lane slices cover every generic shape exactly once with the
right Ninio index, and the committed .inc file is the generator's output."""
import filecmp
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("gen_mfe_blocks", os.path.join(ROOT, "tools", "gen_mfe_blocks.py"))
G = importlib.util.module_from_spec(spec)
spec.loader.exec_module(G)


def test_partitions_cover_each_loop_size_once():
    for S in (1, 2, 4):   # one partition per lanes-per-cell mode
        blocks, load = G.partition(S)
        sizes = sorted(u for b in blocks for u in b)
        assert sizes == list(range(G.MAXLOOP + 1))
        assert len(blocks) == G.NBLK and max(load) - min(load) <= 10, (S, load)


def _slice_edges(S, r, u):
    """mfe_cells.hip B setup: slice r's (ea, eb) and the edge n1 it reads."""
    eb = r & 1
    ea = ((-(r >> 1)) if (r & 1) else (r >> 1)) if S == 4 else (-1 if (r & 1) else 1)
    return [ea + eb * u] if S == 4 else [eb * u, ea + eb * u]


def test_sliced_edge_shapes_once_per_cell():
    """Sizes u >= 4 read their bulges and 1 x n loops on one slice each (4 lanes
    per cell) or two per slice (2 lanes per cell); the kinds match the table the
    slice uses (CT_BUL on slices 0, 1, CT_ONEN on 2, 3)."""
    for u in range(4, G.MAXLOOP + 1):
        for S in (2, 4):
            got = sorted(n for r in range(S) for n in _slice_edges(S, r, u))
            assert got == sorted(G.edges(u)), (S, u, got)
        for r in range(4):
            (n1,) = _slice_edges(4, r, u)
            assert G.kind(n1, u - n1) == ("1n" if r & 2 else "bul"), (u, r)
        for r in range(2):
            b, n = _slice_edges(2, r, u)
            assert G.kind(b, u - b) == "bul" and G.kind(n, u - n) == "1n"
        pre, decl, lines, outs, ins, post = G.sliced_parts(u, 4, "a")
        # the edge shapes are not also read at fixed offsets
        fixed = {int(ln.split("offset:")[1]) // 4 for ln in lines if "%[qaa] offset:" in ln}
        assert not fixed & set(G.edges(u)), (u, fixed)


def test_shape_kinds():
    # generic (il[u] + nin[|u1-u2|]) exactly when both sides have >= 2 unpaired
    # bases, except the tabulated 2x2 and 2x3 / 3x2 loops (oracle/fold.c E_int)
    for u in range(G.MAXLOOP + 1):
        for u1 in range(u + 1):
            u2 = u - u1
            gen = min(u1, u2) >= 2 and (min(u1, u2), max(u1, u2)) not in ((2, 2), (2, 3))
            assert (G.kind(u1, u2) == "gen") == gen


def test_sliced_generic_coverage():
    for S in (2, 4):
        for u in range(G.MAXLOOP + 1):
            gen = [u1 for u1 in range(u + 1) if G.kind(u1, u - u1) == "gen"]
            if not gen:
                continue
            nk = (len(gen) + S - 1) // S
            seen = [gen[0] + r + S * k for k in range(nk) for r in range(S) if gen[0] + r + S * k in gen]
            assert sorted(seen) == gen   # each generic shape in exactly one (slice, position)
            pre, decl, lines, outs, ins, post = G.sliced_parts(u, S, "a")
            reads = [ln for ln in lines if "%[qga]" in ln]
            assert len(reads) == nk
            body = "\n".join(post)
            for k in range(nk):   # every position is folded: with its energy or on the plateau
                assert "w%da" % k in body


def test_committed_blocks_match_generator(tmp_path):
    env = dict(os.environ, ADX_GEN_OUT=str(tmp_path))
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gen_mfe_blocks.py")], env=env,
                          stderr=subprocess.DEVNULL)
    for name in ("mfe_blocks.inc", "mfe_pair_blocks.inc"):
        assert filecmp.cmp(str(tmp_path / name), os.path.join(ROOT, "addapt_amd", "csrc", name), shallow=False), name


def test_pair_partitions_skip_stack_and_bulge1():
    """The pair kernel's blocks hold loop sizes 2..30 once each (the stack and
    bulge-1 shapes run in its finalize, mfe_pair.hip) and add the per-lane
    diagonal offset hb * u to every inner-cell address."""
    G.PAIR = True
    try:
        for S in (1, 2, 4):
            blocks, load = G.partition(S)
            assert sorted(u for b in blocks for u in b) == list(range(2, G.MAXLOOP + 1)), S
        pre = G.sliced_parts(17, 4, "a")[0]
        assert "off(dd - 19, U.N) + ci + hb * 17" in pre[0]
    finally:
        G.PAIR = False
