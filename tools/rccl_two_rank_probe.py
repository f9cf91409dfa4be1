"""Probe: can two processes on ONE GPU form an RCCL communicator through the
product ABI (cgpu_comm_init) and sum their delta buffers
(cgpu_counters_allreduce)?  RCCL normally refuses two ranks on one device
("Duplicate GPU detected"); this records what this ROCm build does.

    python tools/rccl_two_rank_probe.py            # parent: spawns 2 ranks
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank: int, idfile: str) -> int:
    import torch
    from cilium_amd.engine import Engine
    e = Engine(device=0)
    e.commit()
    if rank == 0:
        cid = Engine.comm_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(cid)
        os.replace(idfile + ".tmp", idfile)
    else:
        for _ in range(300):
            if os.path.exists(idfile):
                break
            time.sleep(0.1)
        cid = open(idfile, "rb").read()
    try:
        e.comm_init(cid, 2, rank)
    except Exception as ex:  # noqa: BLE001
        print(f"rank {rank}: comm_init failed: {ex}", flush=True)
        return 3
    buf = torch.full((e.counter_delta_bytes() // 8,), rank + 1, dtype=torch.int64, device="cuda")
    e.counter_bind(buf)
    e.counters_allreduce()
    torch.cuda.synchronize()
    ok = bool((buf == 3).all())
    print(f"rank {rank}: allreduce {'ok' if ok else 'WRONG'}", flush=True)
    e.counter_bind(None)
    e.close()
    return 0 if ok else 4


if __name__ == "__main__":
    if len(sys.argv) > 2:
        sys.exit(rank_main(int(sys.argv[1]), sys.argv[2]))
    idfile = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"cgpu_probe_{os.getpid()}.id")
    procs = [subprocess.Popen([sys.executable, __file__, str(r), idfile]) for r in range(2)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=90))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    print(f"two-rank probe exit codes: {rcs}", flush=True)
    sys.exit(0)
