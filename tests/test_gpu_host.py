"""Host-resident batches (cgpu_classify_v4_host): the same tuples
classified from host memory (pageable numpy arrays and page-locked tensors,
several 8M-tuple chunks with a ragged last one; outputs into pageable arrays,
downloaded, or page-locked ones, which the CUs store into except where a
chunk's column is not 16-byte aligned) give exactly the verdicts,
identities, stages, per-entry counters and metrics of cgpu_classify_v4 over
device columns."""
import numpy as np
import pytest

from cilium_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    from cilium_amd import build
    build.build()
    T = synth.make_tables(n_prefixes=20_000, n_identities=500, n_endpoints=4, keys_per_ep=4000)
    t = synth.make_tuples(T, 9_000_001)
    return torch, T, t


def _engine(T):
    from cilium_amd.engine import Engine
    e = Engine(device=0, **T.engine_config())
    synth.load_engine(e, T)
    e.commit()
    return e


def _counters(e, T):
    out = []
    for k, ep in zip(T.pol_keys[::5], T.pol_ep[::5]):
        rc, got = e.policy_lookup(int(ep), k)
        assert rc == 0
        out.append((int(got["packets"]), int(got["bytes"])))
    return out


@pytest.mark.parametrize("pinned", [False, True, "outputs"])
def test_host_batch_equals_device_batch(setup, pinned):
    torch, T, t = setup
    ed, eh = _engine(T), _engine(T)
    out = ed.classify_v4(synth.to_device(t))
    torch.cuda.synchronize()
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    cols = {k: np.ascontiguousarray(t[k], dt) for k, dt in synth.TUPLE_DTYPES.items() if k in t}
    if pinned:
        cols = {k: torch.from_numpy(v.view(view[v.dtype.type])).pin_memory() for k, v in cols.items()}
    hout = None
    if pinned == "outputs":
        hout = {k: torch.empty(len(t["saddr"]), dtype=dt).pin_memory()
                for k, dt in (("verdict", torch.int32), ("identity", torch.int32), ("stage", torch.uint8))}
        hout["identity"][:] = -1
    got = eh.classify_v4_host(cols, out=hout)
    if hout is not None:
        torch.cuda.synchronize()
        got = {"verdict": hout["verdict"].numpy(), "identity": hout["identity"].numpy().view(np.uint32),
               "stage": hout["stage"].numpy()}
    np.testing.assert_array_equal(got["verdict"], out["verdict"].cpu().numpy())
    np.testing.assert_array_equal(got["identity"], out["identity"].cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(got["stage"], out["stage"].cpu().numpy())
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    assert _counters(eh, T) == _counters(ed, T)
    ed.close()
    eh.close()


def test_host_batch_past_staging(setup):
    """A batch longer than the device staging (16 chunks of 8M tuples):
    chunk k + 16 reuses chunk k's buffers once its classify is queued."""
    torch, T, _ = setup
    n = 16 * (1 << 23) + 4097
    t = synth.make_tuples(T, n)
    ed, eh = _engine(T), _engine(T)
    out = ed.classify_v4(synth.to_device(t), stage=False)
    torch.cuda.synchronize()
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    cols = {k: torch.from_numpy(np.ascontiguousarray(t[k], dt).view(view[dt])).pin_memory()
            for k, dt in synth.TUPLE_DTYPES.items() if k in t}
    del t
    hout = {k: torch.empty(n, dtype=torch.int32).pin_memory() for k in ("verdict", "identity")}
    hout["stage"] = None
    eh.classify_v4_host(cols, out=hout)
    torch.cuda.synchronize()
    assert torch.equal(hout["verdict"], out["verdict"].cpu())
    assert torch.equal(hout["identity"], out["identity"].cpu())
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    ed.close()
    eh.close()


@pytest.fixture(scope="module")
def config2():
    """BASELINE config 2's tables (100k IPv4 prefixes, 64k policy keys) and
    their restatement, shared by the restatement checks below."""
    import torch
    assert torch.cuda.is_available(), "GPU test needs a device"
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle"))
    from oracle import Oracle
    T = synth.make_tables(**synth.CONFIGS["gpu"])
    o = Oracle(**T.oracle_config())
    synth.load_oracle(o, T)
    return torch, T, o


def _pin(torch, cols):
    view = {np.uint32: np.int32, np.uint16: np.int16, np.uint8: np.uint8}
    return {k: torch.from_numpy(np.ascontiguousarray(v).view(view.get(v.dtype.type, v.dtype))).pin_memory()
            for k, v in cols.items()}


def test_host_batch_vs_restatement_config2(config2):
    """Config-2 tables, 9M + 4097 tuples from page-locked memory (two
    chunks, a ragged last one): verdicts, identities, stages and metrics
    equal the CPU restatement's (oracle/cgpu_oracle.c, pinned to the
    reference's golden vectors); the staging is reported and released."""
    torch, T, o = config2
    n = 9 * (1 << 20) + 4097
    t = synth.make_tuples(T, n, gpu_id=3)
    e = _engine(T)
    cols = _pin(torch, {k: np.ascontiguousarray(t[k], dt) for k, dt in synth.TUPLE_DTYPES.items()
                        if k in t})
    got = e.classify_v4_host(cols)
    o.counters_reset()
    v, idt, st, _ = o.classify_v4(t, nthreads=16)
    np.testing.assert_array_equal(got["verdict"], v)
    np.testing.assert_array_equal(got["identity"], idt)
    np.testing.assert_array_equal(got["stage"], st)
    np.testing.assert_array_equal(e.metrics(), o.metrics())
    assert e.host_stage_bytes() > 0
    e.host_stage_release()
    assert e.host_stage_bytes() == 0
    # the staging comes back on the next host call
    again = e.classify_v4_host({k: x[:5000] for k, x in cols.items()})
    np.testing.assert_array_equal(again["verdict"], v[:5000])
    e.close()


@pytest.mark.parametrize("stride", [64, 128])
@pytest.mark.parametrize("pinned", [True, False])
def test_frames_host_vs_device_and_restatement(config2, stride, pinned):
    """cgpu_classify_frames_host: raw frames of every class in host memory
    (page-locked: read by the CUs; pageable: copied), several chunks with a
    ragged last one, against cgpu_classify_frames over the same frames in
    device memory and against the restatement: verdicts, identities, stages,
    metrics and per-entry counters."""
    torch, T, _ = config2
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_frames_golden import frame_oracle
    from cilium_amd import layouts as L
    from cilium_amd.engine import Engine
    rng = np.random.Generator(np.random.PCG64(0x40F7 + stride))
    pool = T.pfx_addr.astype(np.uint32).byteswap()
    n = 4 * (1 << 20) + 333 if stride == 64 else 2 * (1 << 20) + 77  # two chunks each
    f = synth.make_frames(rng, n, width=stride, n_ep=T.n_endpoints, addr4=pool)
    info = L.lxc_info(synth.LXC_MAC, synth.LXC_IPV4_RAW, synth.LXC_IP6, 7)

    def engine():
        e = Engine(device=0, ct_proto_gate=1, **T.engine_config())
        for ep in range(T.n_endpoints):
            assert e.lxc_update(ep, info) == 0
        synth.load_engine(e, T)
        e.commit()
        return e
    ed, eh = engine(), engine()
    dout = ed.classify_frames(synth.frames_to_device(f))
    torch.cuda.synchronize()
    hf = {"data": np.ascontiguousarray(f["data"]), "len": np.ascontiguousarray(f["len"], np.uint32),
          "flags": np.ascontiguousarray(f["flags"], np.uint8), "ep": np.ascontiguousarray(f["ep"], np.uint16)}
    if pinned:
        hf = {"data": torch.from_numpy(hf["data"]).pin_memory(),
              "len": torch.from_numpy(hf["len"].view(np.int32)).pin_memory(),
              "flags": torch.from_numpy(hf["flags"]).pin_memory(),
              "ep": torch.from_numpy(hf["ep"].view(np.int16)).pin_memory()}
    got = eh.classify_frames_host(hf)
    np.testing.assert_array_equal(got["verdict"], dout["verdict"].cpu().numpy())
    np.testing.assert_array_equal(got["identity"], dout["identity"].cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(got["stage"], dout["stage"].cpu().numpy())
    np.testing.assert_array_equal(eh.metrics(), ed.metrics())
    assert _counters(eh, T) == _counters(ed, T)
    o = frame_oracle(1, 7, n_ep=T.n_endpoints, **T.oracle_config())
    synth.load_oracle(o, T)
    ov, oi, ost, _ = o.classify_frames(f, nthreads=16)
    np.testing.assert_array_equal(got["verdict"], ov)
    np.testing.assert_array_equal(got["identity"], oi)
    np.testing.assert_array_equal(got["stage"], ost)
    np.testing.assert_array_equal(eh.metrics(), o.metrics())
    ed.close()
    eh.close()
