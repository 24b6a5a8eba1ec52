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
    blocks, load = G.partition()
    sizes = sorted(u for b in blocks for u in b)
    assert sizes == list(range(G.MAXLOOP + 1))
    assert len(blocks) == G.NBLK and max(load) - min(load) <= 10


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
    name = "mfe_blocks.inc"
    assert filecmp.cmp(str(tmp_path / name), os.path.join(ROOT, "addapt_amd", "csrc", name), shallow=False), name
