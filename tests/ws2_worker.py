"""One rank of tests/test_gpu_multigpu_ws2.py (not a test module): the
product's exchange glue -- multigpu.merge_cells / merge_grouped with the device
operations (DeviceOps) -- between separate processes on one GPU over gloo,
whose device-tensor collectives multigpu stages through host memory.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p \\
        python tests/ws2_worker.py OUT.npz N MODE     MODE: cells | wide | g<users>
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import torch.distributed as dist

    from heatmap_amd import device, multigpu, synth

    out, n, mode = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    per = n // ws
    lat, lon = synth.generate("hotspots", per, seed=11, start=rank * per)
    if mode in ("cells", "wide"):
        m, buf = device.count_device(lat, lon, None, 0, 18)
        widek = -1
        if mode == "wide" and rank == ws - 1:
            # one sparse cell's count past 2^32: its route flags HM_E_WIDE, the
            # flag rides on the size exchange and every rank routes again with
            # int64 counts
            i = int(torch.nonzero((buf.keys[:m] >> 58) > 10)[0, 0])
            buf.counts[i] += 1 << 32
            widek = int(buf.keys[i])
        own = multigpu.merge_cells(buf, m, ws, rank, dense_zmax=10)
        torch.cuda.synchronize()
        np.savez(out, keys=buf.keys[:own].cpu().numpy(), counts=buf.counts[:own].cpu().numpy(),
                 widek=np.int64(widek), nx=np.int64(buf.nx))
    else:
        users = int(mode[1:])
        grp = ((np.arange(rank * per, (rank + 1) * per) * 2654435761) >> 7) % users
        k, gc = device.count_grouped_packed_device(lat, lon, grp.astype(np.uint32), None, 6, 21)
        hk, g, c = multigpu.merge_grouped(k, gc, ws, rank)
        torch.cuda.synchronize()
        np.savez(out, keys=hk.cpu().numpy(), groups=g.cpu().numpy(), counts=c.cpu().numpy())
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
