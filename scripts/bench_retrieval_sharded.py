"""Gallery-sharded retrieval at the BASELINE configs' dataset sizes.

BASELINE.json configs[3] is "CUHK03-detected ResNet-50 PPS, 4xMI355X
gallery-sharded, RCCL all-gather over xGMI": Q = 1400, G = 5332.
This runs bench.py's retrieval stage (distance block on each rank's gallery
shard + count-based mAP/CMC) at those sizes, one process per GPU:

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
      --master-addr 127.0.0.1 --master-port 29511 \
      scripts/bench_retrieval_sharded.py --dataset cuhk03

With PPS_DIST_BACKEND=gloo the same ranks share the GPUs there are (a
one-GPU rehearsal: timings are then not per-GPU figures, but mAP/CMC must
equal the single-rank run's exactly).  Synthetic features (SURVEY §8(d)
recipe), since there are no datasets on the box.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# (queries, gallery, id-0 distractors in the gallery, identities)
DATASETS = {
    'market1501': (3368, 15913, 2793, 750),
    'cuhk03': (1400, 5332, 0, 700),      # detected, new protocol
    'duke': (2228, 17661, 0, 1110),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dataset', default='cuhk03', choices=sorted(DATASETS))
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    backend = os.environ.get('PPS_DIST_BACKEND', 'nccl')
    if backend == 'gloo':
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    from pps_amd import distributed as pdist
    nq, ng, ndis, nids = DATASETS[args.dataset]
    ret = bench.retrieval_stage(rank, world, args.reps, tune=True, nq=nq, ng=ng,
                                n_distractors=ndis, n_ids=nids)
    d = bench.D_FEAT
    dist_ms = pdist.max_over_ranks(ret['distmat_ms'], world)
    total_ms = pdist.max_over_ranks(ret['retrieval_ms'], world)
    total_bytes = (nq + ng) * d * 4 + nq * ng * 4
    if rank == 0:
        print(json.dumps({
            'workload': '%s retrieval, %dq x %dg, D=%d, L2, gallery-sharded over %d rank(s)'
                        % (args.dataset, nq, ng, d, world),
            'backend': backend if world > 1 else 'none', 'n_ranks': world,
            'G_local_rank0': ret['G_local'],
            'distmat_ms': round(dist_ms, 3),
            'distmat_GBps': round(total_bytes / (dist_ms * 1e-3) / 1e9, 2),
            'distmat_TFLOPs_rank0': round(2.0 * nq * ret['G_local'] * d
                                          / (ret['distmat_ms'] * 1e-3) / 1e12, 2),
            'retrieval_ms': round(total_ms, 3),
            'distmat_tile': ret['distmat_tile'], 'distmat_qplanes': ret['distmat_qplanes'],
            'mAP': round(ret['mAP'], 9), 'cmc1': ret['cmc1'], 'cmc5': ret['cmc5'],
            'cmc10': ret['cmc10']}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
