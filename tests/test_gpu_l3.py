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


def random_workload(seed):
    from cilium_amd import synth
    return synth.make_l3_workload(n_rules=400, n_endpoints=24, n_identities=3000, seed=seed)


@pytest.mark.parametrize("flags", [3, 1, 0])
def test_l3_random_vs_restatement(engine, flags):
    repo, eps, ids = random_workload(42 + flags)
    prog = repo.compile()
    got = engine.l3_compile(prog, eps, ids, flags)
    ref = Oracle.l3_compile(prog, eps, ids, flags)
    np.testing.assert_array_equal(got, ref)
    if flags == 3:  # the random repository exercises both outcomes
        assert (got & 1).any() and not (got & 1).all()
