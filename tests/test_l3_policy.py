"""L3 MapState compilation.

CPU: the restatement (oracle/cgpu_oracle.c or_l3_compile) over the tables
cilium_amd/policy.py compiles, pinned to the decisions the reference's own
Go tests assert (tests/golden/l3_policy_cases.json: repository_test.go
TestCanReachIngress / TestCanReachEgress, rule_test.go TestRuleCanReach),
plus the label / selector semantics of pkg/labels and the k8s requirement
operators.  Go is not in this image, so no other reference output exists:
cases beyond those are "parity unpinned" against the reference and checked
GPU-vs-restatement only (tests/test_gpu_l3.py)."""
import json
import os

import numpy as np
import pytest

from cilium_amd import policy as P
from oracle import Oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "l3_policy_cases.json")


def _sel(spec):
    if isinstance(spec, list):
        return P.EndpointSelector.from_labels(*[P.parse_select_label(s) for s in spec])
    return P.EndpointSelector(spec.get("match_labels", {}),
                              [tuple(x) for x in spec.get("expr", [])])


def build_repo(rules):
    repo = P.Repository()
    for r in rules:
        repo.add(P.Rule(
            _sel(r["subject"]),
            [P.IngressRule([_sel(s) for s in i.get("from_requires", [])],
                           [_sel(s) for s in i.get("from_endpoints", [])], i.get("to_ports", False))
             for i in r.get("ingress", [])],
            [P.EgressRule([_sel(s) for s in e.get("to_requires", [])],
                          [_sel(s) for s in e.get("to_endpoints", [])], e.get("to_ports", False))
             for e in r.get("egress", [])]))
    return repo


def decide(prog, ctx_from, ctx_to, direction, flags=3):
    """One SearchContext: ingress asks (endpoint = To, identity = From),
    egress (endpoint = From, identity = To)."""
    if direction == "ingress":
        a = Oracle.l3_compile(prog, [ctx_to], [ctx_from], flags)[0, 0] & 1
    else:
        a = Oracle.l3_compile(prog, [ctx_from], [ctx_to], flags)[0, 0] & 2
    return "Allowed" if a else "Denied"


def cases():
    return json.load(open(GOLDEN))["cases"]


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_reference_known_answers(case):
    prog = build_repo(case["rules"]).compile()
    for ch in case["checks"]:
        got = decide(prog, P.parse_select_label_array(*ch["from"]),
                     P.parse_select_label_array(*ch["to"]), ch["dir"])
        assert got == ch["expect"], ch


def test_label_parsing_semantics():
    # labels.go:605-637
    assert P.parse_label("k8s:app=web") == P.Label("k8s", "app", "web")
    assert P.parse_label("app=web") == P.Label("unspec", "app", "web")
    assert P.parse_select_label("app=web") == P.Label("any", "app", "web")
    assert P.parse_label("reserved:host") == P.Label("reserved", "host", "")
    assert P.parse_label("$host") == P.Label("reserved", "host", "")
    assert P.parse_label("reserved.world") == P.Label("reserved", "world", "")


def test_selector_operators_and_sources():
    """Requirement.Matches In / NotIn / Exists / DoesNotExist, the any
    source, source-qualified keys, first-label Get, reserved.all."""
    ident = [P.parse_label("k8s:app=web"), P.parse_label("k8s:tier=fe"),
             P.parse_label("container:app=other")]
    ep = [P.parse_select_label("role=db")]

    def allowed(sel, requires=None):
        repo = P.Repository()
        repo.add(P.Rule(P.EndpointSelector.from_labels(P.parse_select_label("role=db")),
                        [P.IngressRule([requires] if requires else [], [sel])]))
        return bool(Oracle.l3_compile(repo.compile(), [ep], [ident])[0, 0] & 1)

    S = P.EndpointSelector
    assert allowed(S({"k8s.app": "web"}))
    assert not allowed(S({"container.app": "web"}))
    assert allowed(S({"container.app": "other"}))
    assert allowed(S({"any.app": "web"}))            # first label with key app
    assert not allowed(S({"any.app": "other"}))      # Get returns the first one
    assert allowed(S({}, [("any.tier", "In", ["fe", "be"])]))
    assert not allowed(S({}, [("any.tier", "NotIn", ["fe"])]))
    assert allowed(S({}, [("any.zone", "NotIn", ["a"])]))  # absent key
    assert allowed(S({}, [("k8s.tier", "Exists", [])]))
    assert not allowed(S({}, [("k8s.tier", "DoesNotExist", [])]))
    assert allowed(S({"reserved.all": ""}))
    assert not allowed(S({"reserved.all": ""}), requires=S({"any.nope": ""}))
    # an L4-restricted FromEndpoints defers to the L4 stage: not an L3 allow
    repo = P.Repository()
    repo.add(P.Rule(S.from_labels(P.parse_select_label("role=db")),
                    [P.IngressRule([], [S({"k8s.app": "web"})], to_ports=True)]))
    assert Oracle.l3_compile(repo.compile(), [ep], [ident])[0, 0] & 1 == 0
    # enforcement disabled in a direction = allow-all (policy.go:351-389)
    assert Oracle.l3_compile(repo.compile(), [ep], [ident], flags=0)[0, 0] == 3
