"""GPU parity of the L3 MapState compilation:
cgpu_l3_compile against the reference's Go-test known answers and against
the restatement (or_l3_compile) on a large random repository.  Bit-exact."""
import numpy as np
import pytest

from cilium_amd import build, policy as P
from oracle import Oracle

from test_l3_policy import build_repo, cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    build.build()
    from cilium_amd.engine import Engine
    e = Engine(device=0)
    yield e
    e.close()


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_l3_known_answers_gpu(engine, case):
    prog = build_repo(case["rules"]).compile()
    for ch in case["checks"]:
        fr = P.parse_select_label_array(*ch["from"])
        to = P.parse_select_label_array(*ch["to"])
        if ch["dir"] == "ingress":
            a = engine.l3_compile(prog, [to], [fr])[0, 0] & 1
        else:
            a = engine.l3_compile(prog, [fr], [to])[0, 0] & 2
        assert ("Allowed" if a else "Denied") == ch["expect"], ch


def random_repo(rng, n_rules=400, n_keys=12, n_vals=6):
    keys = [f"k{i}" for i in range(n_keys)]
    srcs = ["k8s", "container", "any"]

    def sel(lo=0):
        ml = {}
        for _ in range(rng.integers(lo, 3)):
            ml[f"{rng.choice(srcs)}.{rng.choice(keys)}"] = f"v{rng.integers(0, n_vals)}"
        ex = []
        for _ in range(rng.integers(0, 2)):
            op = str(rng.choice(["In", "NotIn", "Exists", "DoesNotExist"]))
            vals = [f"v{x}" for x in rng.integers(0, n_vals, rng.integers(1, 3))] if op in (
                "In", "NotIn") else []
            ex.append((f"{rng.choice(srcs)}.{rng.choice(keys)}", op, vals))
        if rng.random() < 0.02:
            ml["reserved.all"] = ""
        return P.EndpointSelector(ml, ex)

    repo = P.Repository()
    for _ in range(n_rules):
        ing = [P.IngressRule([sel(1) for _ in range(1 if rng.random() < 0.03 else 0)],
                             [sel(1) for _ in range(rng.integers(0, 3))], bool(rng.random() < 0.2))
               for _ in range(rng.integers(0, 3))]
        eg = [P.EgressRule([sel(1) for _ in range(1 if rng.random() < 0.03 else 0)],
                           [sel(1) for _ in range(rng.integers(0, 3))], bool(rng.random() < 0.2))
              for _ in range(rng.integers(0, 3))]
        repo.add(P.Rule(sel(1), ing, eg))
    return repo, keys, srcs, n_vals


def random_sets(rng, n, keys, srcs, n_vals):
    out = []
    for _ in range(n):
        out.append([P.Label(str(rng.choice(srcs[:2])), str(rng.choice(keys)),
                            f"v{rng.integers(0, n_vals)}") for _ in range(rng.integers(1, 6))])
    return out


@pytest.mark.parametrize("flags", [3, 1, 0])
def test_l3_random_vs_restatement(engine, flags):
    rng = np.random.Generator(np.random.PCG64(42 + flags))
    repo, keys, srcs, nv = random_repo(rng)
    prog = repo.compile()
    eps = random_sets(rng, 24, keys, srcs, nv)
    ids = random_sets(rng, 3000, keys, srcs, nv)
    got = engine.l3_compile(prog, eps, ids, flags)
    ref = Oracle.l3_compile(prog, eps, ids, flags)
    np.testing.assert_array_equal(got, ref)
    if flags == 3:  # the random repository exercises both outcomes
        assert (got & 1).any() and not (got & 1).all()
