#!/usr/bin/env python
"""Can two RCCL ranks share ONE GPU? (run the RCCL data-parallel instance
at world 2 on a one-GPU box.) Spawns two child processes, both on cuda:0:

  1. kdl._C.RcclComm (the native communicator DpLeader / DpFollower use) at world 2, then one
     1 KB rccl_gather;
  2. torch.distributed "nccl" (RCCL) all_reduce at world 2.

Prints what each rank saw (the refusal text if RCCL refuses duplicate devices).
  python tools/probes/rccl_dup_probe.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")


def child(rank: int, idfile: str, port: str) -> int:
    sys.path.insert(0, ROOT)
    import torch
    torch.cuda.set_device(0)
    from kdl.ops import _lib
    C = _lib.lib()
    if rank == 0:
        uid = C.rccl_unique_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile) and time.time() - t0 < 30:
            time.sleep(0.05)
        uid = open(idfile, "rb").read()
    try:
        comm = C.RcclComm(uid, 2, rank, 0)
        send = torch.full((256,), float(rank + 1), device="cuda")
        recv = torch.zeros(512, device="cuda")
        s = torch.cuda.current_stream()
        comm.gather(send.data_ptr(), recv.data_ptr(), 1024, s.cuda_stream)
        torch.cuda.synchronize()
        print(f"rank {rank}: native RcclComm world 2 on one GPU OK; gather block 1 = {recv[256:258].tolist()}",
              flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: native RcclComm REFUSED: {type(e).__name__}: {e}", flush=True)
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        dist.init_process_group("nccl", rank=rank, world_size=2)
        t = torch.ones(4, device="cuda") * (rank + 1)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        print(f"rank {rank}: torch.distributed nccl world 2 on one GPU OK: {t.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: torch.distributed nccl REFUSED: {type(e).__name__}: {str(e)[:400]}", flush=True)
    return 0


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        return child(int(sys.argv[2]), sys.argv[3], sys.argv[4])
    d = tempfile.mkdtemp()
    idfile = os.path.join(d, "uid")
    port = str(29500 + os.getpid() % 1000)
    env = dict(os.environ, NCCL_DEBUG="WARN")
    kids = [subprocess.Popen([sys.executable, __file__, "child", str(r), idfile, port], env=env) for r in range(2)]
    rc = 0
    for k in kids:
        try:
            rc |= k.wait(timeout=120)
        except subprocess.TimeoutExpired:
            print("probe: a rank hung (120 s); killing it", flush=True)
            k.kill()
            rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(main())
