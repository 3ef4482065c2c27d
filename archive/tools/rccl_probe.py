#!/usr/bin/env python3
"""tools/rccl_probe.py -- bench.py's RCCL plumbing on a one-GPU box (tools probe, not
product).  RCCL refuses two ranks on one card, so the N>1 nccl path cannot be rehearsed
there; this runs it at one rank instead, under torch.distributed.run:

  python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port P tools/rccl_probe.py

It does what every bench.py rank does with backend nccl: set the device, eager
init_process_group("nccl", device_id=...), load libcocytus_ec next to RCCL, one encode,
barrier, all_reduce(MAX) of float64 scalars on the device, barrier, destroy."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    init_s = time.perf_counter() - t0
    torch.empty(1, device="cuda")
    from cocytus_amd import ec

    assert ec.device_check() == ec.CEC_OK, ec.lib().cec_last_error().decode()
    k, m, n = 3, 2, 1 << 20
    data = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda") for _ in range(k)]
    par = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    stream = torch.cuda.current_stream()
    ec.encode_region(k, m, ec.coding_matrix(k, m), data, par, n, stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(par[0], data[0] ^ data[1] ^ data[2]))  # row K is all ones
    t1 = time.perf_counter()
    dist.barrier()
    t = torch.tensor([1.5, float(dist.get_rank())], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    coll_ms = (time.perf_counter() - t1) * 1e3
    got = t.tolist()
    dist.destroy_process_group()
    print(json.dumps({"rccl_probe": True, "world": int(os.environ.get("WORLD_SIZE", "1")),
                      "backend": "nccl", "init_s": round(init_s, 3), "collectives_ms": round(coll_ms, 3),
                      "all_reduce_max": got, "encode_ok": ok,
                      "ipc_mode_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}), flush=True)
    return 0 if ok and got[0] == 1.5 else 1


if __name__ == "__main__":
    sys.exit(main())
