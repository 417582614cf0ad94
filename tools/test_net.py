#!/usr/bin/env python
"""Test a PPS re-ID network on MI355X -- same command line as the reference's
tools/test_net.py:49-117 (`--cfg`, `--wait`, `--vis`, `--multi-gpu-testing`,
`--range s e`, trailing KEY VALUE config overrides).

Multi-GPU: launch one process per GPU with torch.distributed.run, e.g.
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
      tools/test_net.py --cfg X --multi-gpu-testing TEST.WEIGHTS w.npz
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_args(argv=None):
    p = argparse.ArgumentParser(description='Test a PPS re-ID network (MI355X)')
    p.add_argument('--cfg', dest='cfg_file', default=None, type=str)
    p.add_argument('--wait', dest='wait', default=True, type=lambda s: s != 'False')
    p.add_argument('--vis', dest='vis', action='store_true')
    p.add_argument('--multi-gpu-testing', dest='multi_gpu_testing', action='store_true')
    p.add_argument('--range', dest='range', default=None, type=int, nargs=2)
    p.add_argument('--trusted-weights', action='store_true',
                   help='allow unpickling a Detectron .pkl weights file')
    p.add_argument('opts', default=None, nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    import torch
    from pps_amd import config, test_engine
    if args.cfg_file is not None:
        config.merge_cfg_from_file(args.cfg_file)
    if args.opts:
        config.merge_cfg_from_list(args.opts)
    cfg = config.assert_and_infer_cfg()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    # JPEG decode processes, forked from a server started before this process
    # touches the GPU (pps_amd/decode_pool.py); the CPUs split over the ranks
    from pps_amd import decode_pool
    decode_pool.start(decode_pool.default_workers(
        share=int(os.environ.get('LOCAL_WORLD_SIZE', world))))
    if world > 1:
        local = int(os.environ.get('LOCAL_RANK', '0'))
        torch.cuda.set_device(local)
        torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', local))
    while not os.path.exists(cfg.TEST.WEIGHTS) and args.wait:
        print("Waiting for '{}' to exist...".format(cfg.TEST.WEIGHTS), flush=True)
        time.sleep(60)
    res = test_engine.run_inference(
        cfg.TEST.WEIGHTS, ind_range=args.range,
        multi_gpu_testing=args.multi_gpu_testing or world > 1,
        check_expected_results=True, trusted=args.trusted_weights)
    if args.range is None and (world == 1 or torch.distributed.get_rank() == 0):
        print(json.dumps(res))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
