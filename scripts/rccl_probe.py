"""RCCL rehearsal on a 1-GPU box: N ranks share cuda:0 (backend nccl).

Checks the tensor collectives the framework issues (all_reduce, in-place
reduce_scatter_tensor / all_gather_into_tensor with AVG, broadcast, p2p) and
prints one line per rank.  Launch: python scripts/rccl_probe.py N
"""
import os
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=r, world_size=n,
                            device_id=torch.device("cuda", 0))
    x = torch.full((1 << 20,), float(r + 1), device="cuda")
    dist.all_reduce(x)
    assert torch.all(x == n * (n + 1) / 2), x[:4]
    buf = torch.arange(n * 1024, dtype=torch.float32, device="cuda") + r
    shard = buf.view(n, -1)[r]
    dist.reduce_scatter_tensor(shard, buf, op=dist.ReduceOp.AVG)
    want = torch.arange(n * 1024, dtype=torch.float32, device="cuda").view(n, -1)[r] + (n - 1) / 2
    assert torch.allclose(shard, want), (shard[:4], want[:4])
    dist.all_gather_into_tensor(buf, shard)
    assert torch.allclose(buf.view(n, -1)[0],
                          torch.arange(1024, dtype=torch.float32, device="cuda") + (n - 1) / 2)
    if n > 1:
        t = torch.full((4,), float(r), device="cuda")
        if r == 0:
            dist.send(t + 10, dst=1)
        elif r == 1:
            dist.recv(t, src=0)
            assert torch.all(t == 10)
    torch.cuda.synchronize()
    dist.barrier()
    print(f"rank {r}/{n} rccl ok", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        child()
    else:
        n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
        ps = [subprocess.Popen([sys.executable, "-u", __file__],
                               env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(n),
                                        MASTER_ADDR="127.0.0.1", MASTER_PORT="29611"))
              for r in range(n)]
        sys.exit(max(p.wait() for p in ps))
