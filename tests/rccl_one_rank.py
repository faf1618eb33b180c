"""One-rank RCCL run of reticulum_amd.shard's device-tensor branches (driven
by tests/test_rccl_one_rank_gpu.py in a child process, so the process group
never outlives it).  On a one-GPU box RCCL refuses two ranks on one device,
so these branches otherwise first run inside the driver's multi-GPU bench;
one rank still goes through ncclCommInitRank with device_id, a broadcast of
an HBM key table, barriers (an all-reduce on the device), the pipelined
sharded call, and a grouped self send/recv of device tensors through
shard._Posted.  Prints one JSON line of results; rank-0 checks against the
C oracle are made by the parent test."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import datetime
    import torch
    import torch.distributed as dist
    from reticulum_amd import device, shard

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=60))
    out["backend"] = dist.get_backend()
    g = torch.Generator().manual_seed(11)
    keys = torch.randint(0, 256, (300, 64), dtype=torch.uint8, generator=g)
    table = shard.broadcast_keys(keys.to(dev), src=0, device=dev)
    out["table_equal"] = bool(torch.equal(table.cpu(), keys))
    ks = shard.broadcast_keyset(keys.to(dev), src=0, device=dev)
    n, L = 1000, 200
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, generator=g)
    kidx = torch.randint(0, 300, (n,), dtype=torch.int32, generator=g)
    tl = 16 + 16 * (L // 16 + 1) + 32
    tok = torch.empty((n, tl), dtype=torch.uint8, device=dev)
    device.encrypt_uniform(ks, pt.to(dev), L, iv.to(dev), tok, key_idx=kidx.to(dev))
    torch.cuda.synchronize()
    out["tokens"] = tok.cpu().numpy().tobytes().hex()

    # the pipelined sharded call at one rank (barriers and the size table on
    # RCCL; rank 0's own chunks copied into place)
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L

    def enc_work(b, o, l, rows):
        m = l.numel()
        t = torch.empty((m, tl), dtype=torch.uint8, device=dev)
        device.encrypt_uniform(ks, b.view(m, L), L, rows[0], t, key_idx=rows[1])
        return t.view(-1), None, None, []

    res, _ = shard.sharded_call_pipelined(enc_work, pt.to(dev).view(-1), off, lens, rows=[iv.to(dev), kidx.to(dev)],
                                          row_specs=[(torch.uint8, 16), (torch.int32, 0)],
                                          out_cap=lambda x: x * 0 + tl, chunks=3, device=dev,
                                          sync=torch.cuda.synchronize)
    out["pipelined_equal"] = bool(torch.equal(res[0].view(n, tl), tok))

    # grouped self send/recv of device tensors through shard._Posted
    src = torch.randint(0, 256, (1 << 16,), dtype=torch.uint8, generator=g).to(dev)
    dst = torch.zeros_like(src)
    try:
        p = shard._Posted([("send", src, 0), ("recv", dst, 0)], None)
        p.wait()
        torch.cuda.synchronize()
        out["self_p2p"] = "ok" if torch.equal(src, dst) else "mismatch"
    except Exception as e:     # noqa: BLE001 (recorded: the parent test reports the refusal)
        out["self_p2p"] = f"refused: {type(e).__name__}: {e}"
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
