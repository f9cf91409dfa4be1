"""Host-resident batches (cgpu_classify_v4_host): the same tuples
classified from host memory (pageable numpy arrays and page-locked tensors,
several 4M-tuple chunks with a ragged last one; outputs into pageable arrays,
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
    """A batch longer than the device staging (16 chunks of 4M tuples):
    chunk k + 16 reuses chunk k's buffers once its classify is queued."""
    torch, T, _ = setup
    n = 16 * (1 << 22) + 4097
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
