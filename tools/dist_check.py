"""N-rank rehearsal of the sharded paths on the GPU(s) of one box: each rank
runs its share (Jaccard owner tasks + all-reduce, ApproxER column blocks +
all-gather, metric-backbone source rows + all-reduce) and rank 0 compares the
assembled vectors bit for bit with a single-process run.

  GSPARSE_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \\
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/dist_check.py

Ranks beyond the visible GPUs share them (device = LOCAL_RANK mod count)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-sparsification-research_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    backend = os.environ.get("GSPARSE_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.core import GraphSparsifier
    from gsparse.data import Data
    from gsparse.distributed import Comm, sharded_approx_er, sharded_backbone, sharded_edge_scores
    from gsparse.engine import Engine
    from gsparse.metric_backbone import backbone_mask

    comm = Comm(device=dev)
    ok = True
    for name, ei, n in [("roman", graphs.roman_like(), 22_662),
                        ("rmat14", graphs.rmat(14, 8, seed=5), 1 << 14)]:
        ctx = Context(local)
        ctx.set_graph_edge_index(n, torch.from_numpy(ei[0].copy()).to(dev),
                                 torch.from_numpy(ei[1].copy()).to(dev))
        eng = Engine(ctx)
        jac = sharded_edge_scores(eng, comm, "jaccard").cpu().numpy()
        er = sharded_approx_er(eng, comm, max_cg_iters=60, blas_threads=8).cpu().numpy()
        sp_ = GraphSparsifier(Data(edge_index=torch.from_numpy(ei), num_nodes=n), f"cuda:{local}")
        cost = sp_._scores_to_cost(sp_.compute_scores("jaccard"), "jaccard")[: ei.shape[1]]
        keep = sharded_backbone(comm, ei, n, cost)
        if rank == 0:
            ctx1 = Context(local)
            ctx1.set_graph_edge_index(n, torch.from_numpy(ei[0].copy()).to(dev),
                                      torch.from_numpy(ei[1].copy()).to(dev))
            e1 = Engine(ctx1)
            jac1 = e1.jaccard(0, e1.nnz)
            er1 = e1.approx_er(max_cg_iters=60, blas_threads=8)
            keep1 = backbone_mask(ei, n, cost, 1e-9)
            res = {"jaccard": np.array_equal(jac.view(np.uint64), np.asarray(jac1).view(np.uint64)),
                   "approx_er": np.array_equal(er.view(np.uint64), np.asarray(er1).view(np.uint64)),
                   "backbone": np.array_equal(keep, np.asarray(keep1, dtype=bool))}
            print(f"world={world} {name}: {res}", flush=True)
            ok = ok and all(res.values())
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
