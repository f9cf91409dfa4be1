"""The bench roofline's measured ceilings (profiles/ceilings.json, from
tools/microbench/ceilings.hip on an MI355X) and its composition of a path's
reference map lookups into a time floor (bench.roofline): the floor is a
bound the step cannot beat -- the measured two-tier mixes stay within it and
the fraction of any step no faster than the ceilings is <= 1."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ceil():
    return json.load(open(os.path.join(ROOT, "profiles", "ceilings.json")))


def test_ceilings_measured_and_consistent(ceil):
    g = ceil["gather"]
    assert len(g) >= 10 and g[0][0] <= 16 << 10 and g[-1][0] >= 1 << 30
    assert ceil["device"].get("arch", "").startswith("gfx950")
    assert ceil["atomic_sum_ok"] is True and ceil["atomic_g_per_s"] > 0
    assert ceil["stream"]["read_gbs"] < 8000 and ceil["stream"]["write_gbs"] < 8000
    # the tier envelope never rises with table size
    rates = [bench.tier_rate(ceil, s) for s, _ in g]
    assert all(a >= b for a, b in zip(rates, rates[1:]))
    # L2-resident tables are served several times faster than HBM
    assert bench.tier_rate(ceil, 2 << 20) > 3 * bench.tier_rate(ceil, 4 << 30)


def test_measured_mixes_within_composed_ceiling(ceil):
    assert ceil["mix"], "no measured mixes"
    for m in ceil["mix"]:
        assert m["composed_over_measured"] >= 1.0, m


def test_roofline_composition():
    """One L2-resident map: the floor is lookups / R; a second map in a
    larger table adds a floor of its own; frac <= 1 whenever the step is no
    faster than the ceilings, and the bound names the largest floor."""
    ceil = json.load(open(bench.CEILINGS))
    n = 1 << 26
    tb = {"ipcache": 1 << 20, "policy": 2 << 20, "lb4": 85 << 20, "ct4": 768 << 20}
    r2 = bench.tier_rate(ceil, 1 << 20)
    t = 2 * n / (r2 * 1e9)  # exactly the floor of 2 lookups per tuple
    r = bench.roofline(n, t * 1e3, 18, 8, 2 * n, {"ipcache": n, "policy": n, "lb": 0, "prefilter": 0,
                                                   "endpoint": 0}, tb, False, None)
    assert r["bound"] == "gather" and abs(r["frac"] - 1.0) < 1e-3
    assert r["components"]["atomic"] is None
    # a slower step: the fraction falls with it
    r = bench.roofline(n, 4 * t * 1e3, 18, 8, 2 * n, {"ipcache": n, "policy": n, "lb": 0, "prefilter": 0,
                                                       "endpoint": 0}, tb, False, None)
    assert abs(r["frac"] - 0.25) < 1e-3
    # conntrack operations (probe count minus the per-map split) priced at the
    # CT map's tier: one per tuple in a 768-MiB table dominates
    rc = bench.tier_rate(ceil, 768 << 20)
    r = bench.roofline(n, 1e3 * n / (rc * 1e9), 22, 9, 3 * n, {"ipcache": n, "policy": n, "lb": 0,
                                                               "prefilter": 0, "endpoint": 0},
                       tb, False, None)
    assert r["components"]["gather"]["maps"]["ct"]["table"] == "ct4"
    assert r["components"]["gather"]["binding_table_bytes"] == 768 << 20
    assert r["frac"] <= 1.0 + 1e-3
    # the memory-side atomics of a stamped profile bound a step that issues many
    at = {"memory_side_atomics_per_step": 10 * n}
    r = bench.roofline(n, 1e3 * 10 * n / (ceil["atomic_g_per_s"] * 1e9), 18, 8, n,
                       {"ipcache": n, "policy": 0, "lb": 0, "prefilter": 0, "endpoint": 0}, tb, False, at)
    assert r["bound"] == "atomic" and abs(r["frac"] - 1.0) < 1e-3
