"""AutoScalingThermostat (reference sampling.cc:382-401) in the oracle.

The median is std::nth_element at n/2 and the clamp is std::max(t, 0.0).
Both are pinned here against vectors made by the host libstdc++
(tests/golden/gen_nth_element.cc): the element nth_element leaves at k, bit for
bit (which of +0.0 / -0.0 lands there, NaN placement), and the clamped T.
std::max keeps -0.0 and NaN, so a zero median with rate < 1 gives T = -0.0
and the Metropolis rule (sampling.cc:76-89) then rejects every improvement
and accepts every worsening."""
import json
import math
import os
import struct

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "nth_element.json")


def _d(h):
    return struct.unpack("<d", struct.pack("<Q", int(h, 16)))[0]


def _bits(x):
    return "%016x" % struct.unpack("<Q", struct.pack("<d", x))[0]


def test_nth_element_matches_libstdcxx(oracle):
    cases = json.load(open(GOLD))["cases"]
    assert len(cases) >= 50
    for c in cases:
        vals = [_d(h) for h in c["in"]]
        out = oracle.nth_element(vals, c["k"])
        assert [_bits(x) for x in out] == c["out"], (c["in"][:8], c["k"])
        t = oracle.auto_clamp(out[c["k"]] / math.log(0.5))
        assert _bits(t) == c["T_rate_0.5"]


@pytest.mark.parametrize("t,expect", [(-0.0, "-0"), (0.0, "+0"), (float("nan"), "nan"),
                                      (-1.5, "+0"), (2.0, 2.0)])
def test_clamp_rule(oracle, t, expect):
    T = oracle.auto_clamp(t)  # std::max(t, 0.0)
    if expect == "nan":
        assert math.isnan(T)
    elif expect == "-0":
        assert T == 0.0 and math.copysign(1.0, T) < 0
    elif expect == "+0":
        assert T == 0.0 and math.copysign(1.0, T) > 0
    else:
        assert T == expect


def test_zero_median_gives_negative_zero_T(oracle):
    # +0.0 / ln(0.5) = -0.0, kept by std::max; a NaN median stays NaN
    T = oracle.auto_clamp(0.0 / math.log(0.5))
    assert T == 0.0 and math.copysign(1.0, T) < 0
    assert math.isnan(oracle.auto_clamp(float("nan") / math.log(0.5)))


def _metropolis(diff, T, u):
    # sampling.cc:76-89: REJECT iff exp(diff / T) < u
    with_np = __import__("numpy")
    with with_np.errstate(all="ignore"):
        crit = float(with_np.exp(with_np.float64(diff) / with_np.float64(T)))
    if crit < u:
        return "reject"
    return "improved" if diff > 0 else "worsened"


def test_metropolis_after_negative_zero_T():
    T = -0.0
    assert _metropolis(+0.1, T, 0.3) == "reject"      # exp(-inf) = 0 < u
    assert _metropolis(-0.1, T, 0.3) == "worsened"    # exp(+inf) accepted
    assert _metropolis(0.0, T, 0.3) == "worsened"     # exp(nan): nan < u is false
    Tp = +0.0                                          # the old (t > 0 ? t : 0) rule
    assert _metropolis(+0.1, Tp, 0.3) == "improved"
    assert _metropolis(-0.1, Tp, 0.3) == "reject"


def test_metropolis_after_nan_T():
    T = float("nan")
    for d in (0.1, -0.1, 0.0):
        assert _metropolis(d, T, 0.9) != "reject"


def test_mc_run_zero_median_rejects_improvements(oracle):
    """An oracle MFE run whose training set is mostly exact zeros (mutations
    that change no MFE): once T = -0.0 no scored step with diff > 0 is
    accepted and every scored step with diff < 0 is."""
    from addapt_amd import workloads
    tmpl, active = workloads.synthetic(60)
    sf = oracle.ScoreFunction([("apo", 0, False, 1.0)], aptamer=None, mode="mfe")
    th = oracle.thermostat("auto", rate=0.5, period=4, t0=2.0)
    seqs = workloads.walker_sequences(tmpl, [active], 8)
    neg_zero_scored = 0
    for w in range(8):
        r = oracle.mc_run(sf, seqs[w], [active], th, w, 80)
        assert r["rc"] == 0
        cur = sf.score(seqs[w], [active])[0]
        for s, T in enumerate(r["temperature"]):
            out = r["outcome"][s]
            if out != 2 and T == 0.0 and math.copysign(1.0, T) < 0:
                d = r["proposed_score"][s] - cur
                neg_zero_scored += 1
                if d > 0:
                    assert out == 0, (w, s, d)
                elif d < 0:
                    assert out == 1, (w, s, d)
            cur = r["current_score"][s]
    assert neg_zero_scored > 0
