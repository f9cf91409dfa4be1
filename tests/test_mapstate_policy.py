"""Full MapState, CPU side.

Pins the host mirror of the L4 policy resolution (cilium_amd/policy.py
Repository.resolve_l4, compile_mapstate) and the independent restatement
(oracle/mapstate.py) to the answers the reference's own Go tests assert:
tests/golden/l4_policy_cases.json (repository_test.go, rule_test.go,
l4Filter_test.go) and the CIDR helpers' known answers (pkg/ip/ip_test.go
TestRemoveCIDRs, pkg/labels/cidr/cidr_test.go, pkg/policy/api/cidr_test.go).
Go is not in this image; the MapState keys built from these structures are
checked GPU-vs-restatement in tests/test_gpu_mapstate.py."""
import ipaddress
import json
import os
import sys

import pytest

from cilium_amd import policy as P, synth

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import mapstate as M  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "l4_policy_cases.json")


def sel(spec):
    if isinstance(spec, list):
        return P.EndpointSelector.from_labels(*[P.parse_select_label(s) for s in spec])
    return P.EndpointSelector(dict(spec.get("match_labels", {})),
                              [(k, op, list(v)) for k, op, v in spec.get("expr", [])])


def block(d, ingress):
    pre = "from_" if ingress else "to_"
    kw = {}
    for f in ("endpoints", "requires"):
        if pre + f in d:
            kw[pre + f] = [sel(s) for s in d[pre + f]]
    for f in ("entities", "cidr"):
        if pre + f in d:
            kw[pre + f] = list(d[pre + f])
    if "to_ports" in d:
        kw["to_ports"] = [P.PortRule([tuple(p) for p in pr["ports"]],
                                     [("GET", "/")] if pr.get("http") else [],
                                     [("produce",)] if pr.get("kafka") else [])
                          for pr in d["to_ports"]]
    return (P.IngressRule if ingress else P.EgressRule)(**kw)


def repo_of(rules):
    repo = P.Repository()
    for r in rules:
        repo.add(P.Rule(sel(r["subject"]), [block(b, True) for b in r.get("ingress", [])],
                        [block(b, False) for b in r.get("egress", [])]))
    return repo


def canon(es):
    return (tuple(sorted(es.match_labels.items())),
            tuple((k, {"In": "In"}.get(op, op), tuple(v)) for k, op, v in es.match_expressions))


def cases():
    return json.load(open(GOLDEN))["cases"]


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_l4_known_answers(case):
    repo = repo_of(case["rules"])
    for chk in case["resolve"]:
        ctx = P.parse_select_label_array(*chk["ctx"])
        ingress = chk["dir"] == "ingress"
        wc = case.get("level") != "rule"
        if chk.get("error"):
            with pytest.raises(P.PolicyError):
                repo.resolve_l4(ctx, ingress, wc)
            with pytest.raises(M.L4Error):
                M.resolve_l4(repo.rules, ctx, ingress, wc)
            continue
        got = repo.resolve_l4(ctx, ingress, wc)
        ora = M.resolve_l4(repo.rules, ctx, ingress, wc)
        assert sorted(got) == sorted(chk["expect"]) == sorted(ora)
        for key, exp in chk["expect"].items():
            f, o = got[key], ora[key]
            assert (f.port, f.u8proto, f.parser) == (exp["port"], exp["u8proto"], exp["parser"])
            assert tuple(o[:3]) == (exp["port"], exp["u8proto"], exp["parser"])
            if "endpoints" in exp:  # l4Filter_test's repository cases assert SelectsAllEndpoints only
                want = [canon(sel(s)) for s in exp["endpoints"]]
                assert [canon(s) for s in f.endpoints] == want
                assert [canon(s) for s in o[3]] == want
            assert f.ingress == ingress
        for key, v in chk.get("selects_all", {}).items():
            assert got[key].allows_all() is v


def _nets(*pairs):
    return [(ipaddress.ip_address(a), n) for a, n in pairs]


def test_remove_cidrs_known_answers():
    """pkg/ip/ip_test.go:96-163 TestRemoveCIDRs, outputs in the asserted order"""
    got = P.remove_cidrs(_nets(("10.0.0.0", 8)), _nets(("10.96.0.0", 12), ("10.112.0.0", 13)))
    assert got == _nets(("10.128.0.0", 9), ("10.0.0.0", 10), ("10.64.0.0", 11), ("10.120.0.0", 13))
    got = P.remove_cidrs(_nets(("10.0.0.0", 8)),
                         _nets(("10.96.0.0", 12), ("10.112.0.0", 13), ("10.62.0.33", 32),
                               ("10.93.0.4", 30), ("10.63.0.5", 13)))
    assert got == _nets(
        ("10.128.0.0", 9), ("10.0.0.0", 11), ("10.32.0.0", 12), ("10.48.0.0", 13),
        ("10.120.0.0", 13), ("10.64.0.0", 12), ("10.80.0.0", 13), ("10.88.0.0", 14),
        ("10.94.0.0", 15), ("10.92.0.0", 16), ("10.93.128.0", 17), ("10.93.64.0", 18),
        ("10.93.32.0", 19), ("10.93.16.0", 20), ("10.93.8.0", 21), ("10.93.4.0", 22),
        ("10.93.2.0", 23), ("10.93.1.0", 24), ("10.93.0.128", 25), ("10.93.0.64", 26),
        ("10.93.0.32", 27), ("10.93.0.16", 28), ("10.93.0.8", 29), ("10.93.0.0", 30))
    assert P.remove_cidrs(_nets(("10.0.0.0", 8)), _nets(("fd44:7089:ff32:712b::", 66))) is None
    got = P.remove_cidrs(_nets(("fd44:7089:ff32:712b:ff00::", 64)), _nets(("fd44:7089:ff32:712b::", 66)))
    assert got == _nets(("fd44:7089:ff32:712b:8000::", 65), ("fd44:7089:ff32:712b:4000::", 66))


def _lbl(*ss):
    return sorted(P.parse_label_array(*ss), key=lambda l: (l.source, l.key, l.value))


def _sorted(ls):
    return sorted(ls, key=lambda l: (l.source, l.key, l.value))


def test_cidr_labels_known_answers():
    """pkg/labels/cidr/cidr_test.go:50-140 (node CIDRs 10.0.0.0/16 and
    2001:db8:cafe:0:cab::/96 -> cluster ranges /8 and /64); the reference
    asserts the expected labels are all present (Lacks == {})."""
    v4c, v6c = "10.0.0.0/8", "2001:db8:cafe::/64"
    got = set(P.cidr_identity_labels("192.0.2.3/32", v4c))
    assert set(_lbl("cidr:0.0.0.0/0", "cidr:128.0.0.0/1", "cidr:192.0.0.0/8", "cidr:192.0.2.0/24",
                    "cidr:192.0.2.3/32", "reserved:world")) <= got
    assert P.parse_label("cidr:192.0.2.3/24") not in got
    assert len(got) == 34
    got = set(P.cidr_identity_labels("192.0.2.0/24", v4c))
    assert set(_lbl("cidr:0.0.0.0/0", "cidr:192.0.2.0/24", "reserved:world")) <= got
    assert P.parse_label("cidr:192.0.2.3/32") not in got
    assert P.cidr_identity_labels("0.0.0.0/0", v4c) == _lbl("reserved:world")
    got = set(P.cidr_identity_labels("2001:DB8::1/128", v6c))
    assert set(_lbl("cidr:0--0/0", "cidr:2000--0/3", "cidr:2001--0/16", "cidr:2001-d00--0/24",
                    "cidr:2001-db8--0/32", "cidr:2001-db8--1/128", "reserved:world")) <= got
    got = set(P.cidr_identity_labels("10.0.0.0/16", v4c))
    assert set(_lbl("cidr:0.0.0.0/0", "cidr:10.0.0.0/16", "reserved:cluster")) <= got
    got = set(P.cidr_identity_labels("2001:db8:cafe::cab:4:b0b:0/112", v6c))
    assert set(_lbl("cidr:0--0/0", "cidr:2001-db8-cafe--0/64", "cidr:2001-db8-cafe-0-cab-4--0/96",
                    "cidr:2001-db8-cafe-0-cab-4-b0b-0/112", "reserved:cluster")) <= got


def test_cidr_selectors_known_answers():
    """pkg/policy/api/cidr_test.go:37-110 TestGetAsEndpointSelectors"""
    world = P.EndpointSelector.from_labels(P.parse_select_label("reserved:world"))
    v4w = P.EndpointSelector.from_labels(P.ip_string_to_label("0.0.0.0/0"))
    v6w = P.EndpointSelector.from_labels(P.ip_string_to_label("::/0"))
    other = P.EndpointSelector.from_labels(P.ip_string_to_label("192.168.128.0/24"))
    wl = P.parse_label_array("reserved:world")
    for cidrs, exp in ((["0.0.0.0/0"], [world, v4w]), (["::/0"], [world, v6w]),
                       (["0.0.0.0/0", "::/0", "192.168.128.10/24"], [world, v4w, v6w, other])):
        got = P.cidr_selectors(cidrs)
        assert [canon(s) for s in got] == [canon(s) for s in exp]
        assert any(P.selector_matches(s, wl) for s in got)
    assert P.ip_string_to_label("192.168.128.10/24") == P.parse_label("cidr:192.168.128.0/24")
    assert P.ip_string_to_label("::/0") == P.parse_label("cidr:0--0/0")


def test_entity_selectors_known_answers():
    """pkg/policy/api/entity_test.go:23-70: world / cluster / host match their
    reserved labels only, "all" matches everything"""
    lab = {n: P.parse_label_array("reserved:" + n) for n in ("world", "cluster", "host")}
    for ent in ("world", "cluster", "host"):
        s = P.ENTITY_SELECTORS[ent]
        for n, l in lab.items():
            assert P.selector_matches(s, l) == (n == ent)
            assert M.matches(s, l) == (n == ent)
    assert P.selector_matches(P.ENTITY_SELECTORS["all"], P.parse_label_array("k8s:app=x"))
    assert P.entity_selectors(["world", "bogus"]) == [P.ENTITY_SELECTORS["world"]]


def test_parse_port_like_strconv():
    """strconv.ParseUint(s, 0, 16) as CreateL4Filter uses it (l4.go:156)"""
    for s, v in (("80", 80), ("0x50", 80), ("0120", 80), ("0o120", 80), ("0b1010000", 80),
                 ("65535", 65535), ("65536", 0), ("http", 0), ("0", 0), ("08", 0)):
        assert P._parse_port(s) == v == M._port(s), s


def test_random_resolve_product_vs_restatement():
    """the host mirror's resolve_l4 and the restatement's agree filter by
    filter on a random repository of every rule shape"""
    repo, eps, _ = synth.make_mapstate_workload(n_rules=150, n_endpoints=24, n_identities=10, seed=7)
    n = 0
    for ep in eps:
        for ingress in (True, False):
            a = repo.resolve_l4(ep.labels, ingress)
            b = M.resolve_l4(repo.rules, ep.labels, ingress)
            assert list(a) == list(b)
            for k, f in a.items():
                assert (f.port, f.u8proto, f.parser) == tuple(b[k][:3])
                assert [canon(s) for s in f.endpoints] == [canon(s) for s in b[k][3]]
                n += 1
    assert n > 20


def test_compile_mapstate_spec():
    repo, eps, ids = synth.make_mapstate_workload(n_rules=60, n_endpoints=6, n_identities=50, seed=3)
    m = P.compile_mapstate(repo, eps, ids, always_allow_localhost=False, host_allows_world=True)
    assert m.filters.dtype.itemsize == 20 and len(m.ep_map) == 6 and len(m.identity) == 50
    assert (m.filters["sels_off"] + m.filters["n_sels"] <= len(m.filter_sels)).all()
    assert (m.filter_sels < len(m.prog.selectors)).all()
    for row, (ing, eg) in enumerate(m.l4):
        fl = int(m.ep_flags[row])
        has_red = any(f.is_redirect() for f in list(ing.values()) + list(eg.values()))
        assert bool(fl & P.MS_ALLOW_LOCALHOST) == has_red
        assert fl & P.MS_HOST_ALLOWS_WORLD
        assert len(m.filters[m.filters["endpoint"] == row]) == len(ing) + len(eg)


def test_oracle_sync_semantics():
    cur = {(1, 0, 0, 0): 0, (5, 80, 6, 0): 1234, (6, 0, 0, 1): 0}
    want = {(1, 0, 0, 0): 0, (5, 80, 6, 0): 4321, (7, 0, 0, 0): 0}
    new, st = M.sync(cur, want)
    assert new == want
    assert st == dict(added=1, updated=1, deleted=1, unchanged=1)
