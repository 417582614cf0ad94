"""Test-time driver: images -> features -> retrieval metrics, on MI355X.

Same entry points and signatures as the reference's
detectron/core/test_engine.py:
  run_inference(weights_file, ind_range=None, multi_gpu_testing=False,
                gpu_id=0, check_expected_results=False)          :91-143
  test_net_on_dataset(weights_file, dataset_name, proposal_file,
                      output_dir, multi_gpu=False, gpu_id=0)      :146-181
  test_net(weights_file, dataset_name, proposal_file, output_dir,
           ind_range=None, gpu_id=0)  -> ndarray [N, 3968]          :259-370
  initialize_model_from_cfg(weights_file, gpu_id=0)                 :390-405
and the result dict of task_evaluation.py:54-60,345-359.

MI355X-first differences (SURVEY §3.1 hot loop): the reference runs one image
per RunNet with two host<->device copies per image (test.py:163-185).  Here
decode processes (decode_pool, or threads) decode JPEGs for the next batches
while the GPU runs batch b; each batch
is one pinned-memory H2D copy of the raw uint8 pixels, then the preprocessing
kernel (mean-subtract + bicubic), the ResNet-50 / PPS kernels and the
normalisation run on the device, and features stay in HBM for the
evaluation.  Multi-GPU uses one process per GPU (torch.distributed over RCCL)
instead of subprocess + pickle files (utils/subprocess.py:39-103).
"""
import concurrent.futures as futures
import logging
import os
import time
from collections import OrderedDict

import numpy as np
import torch

from . import decode_pool
from . import distributed as pdist
from . import model as pmodel
from . import native
from . import ops
from . import reid_dataset_evaluator as rde
from .config import cfg
from .json_dataset import JsonDataset
from .weights import check_complete, load_weights

logger = logging.getLogger(__name__)


def get_output_dir(dataset_name, training=False):
    if os.sep in dataset_name:  # a json path used as the dataset name
        dataset_name = os.path.splitext(os.path.basename(dataset_name))[0]
    d = os.path.join(cfg.OUTPUT_DIR, 'test' if not training else 'train', dataset_name)
    os.makedirs(d, exist_ok=True)
    return d


def initialize_model_from_cfg(weights_file, gpu_id=0, trusted=False, blobs=None):
    """test_engine.py:390-405: build the test net and load its weights -- as
    one handle of the whole-network C ABI (pps_model_create; every forward
    is one pps_forward call).  PPS_TILES_FILE: apply a saved autotune table
    (bench.py --tiles-file)."""
    torch.cuda.set_device(gpu_id)
    plan = pmodel.build_plan()
    if blobs is None:
        blobs = load_weights(weights_file, trusted=trusted)
    check_complete(blobs, plan)
    m = native.NativeModel(blobs)
    tf = os.environ.get('PPS_TILES_FILE')
    if tf:
        import json
        with open(tf) as f:
            m.apply_table(json.load(f))
    return m


_decode_bgr = decode_pool.decode_bgr


class BatchFeeder(object):
    """Decode on the host, stage raw pixels in pinned memory, one async H2D
    copy per batch, preprocess on the GPU.  `source(i)` returns image i as a
    uint8 BGR array (a path list uses _decode_bgr).  Given the image `paths`
    and a running decode process pool (decode_pool.start), the decode runs in
    those processes, `depth` batches ahead; otherwise on `workers` threads
    one batch ahead (PIL holds the GIL for most of a small image's decode)."""

    def __init__(self, source, n, batch, workers=8, paths=None, depth=4):
        self.source, self.n, self.batch = source, n, batch
        self.procs = decode_pool.pool() if paths is not None else None
        self.paths, self.depth = paths, depth
        self.pool = None if self.procs is not None else futures.ThreadPoolExecutor(max_workers=workers)
        self.H, self.W = cfg.REID.SCALE[1], cfg.REID.SCALE[0]
        self.means = np.asarray(cfg.PIXEL_MEANS, np.float32).ravel()
        self.copy_stream = torch.cuda.Stream()

    def _decode_batch(self, start):
        idx = range(start, min(start + self.batch, self.n))
        return list(self.pool.map(self.source, idx))

    def _submit_procs(self, start):
        ps = self.paths[start:min(start + self.batch, self.n)]
        per = max(2, -(-len(ps) // max(1, decode_pool.workers())))
        return self.procs.map_async(decode_pool.decode_many,
                                    [ps[i:i + per] for i in range(0, len(ps), per)])

    def _stage(self, ims):
        sizes = [im.size for im in ims]
        offs = np.zeros(len(ims), np.int64)
        offs[1:] = np.cumsum(sizes)[:-1]
        blob = torch.empty(int(sum(sizes)), dtype=torch.uint8, pin_memory=True)
        view = blob.numpy()
        for im, o in zip(ims, offs):
            view[o:o + im.size] = im.ravel()
        meta = torch.from_numpy(np.stack([offs, [im.shape[0] for im in ims],
                                          [im.shape[1] for im in ims]])).pin_memory()
        with torch.cuda.stream(self.copy_stream):
            dblob = blob.to('cuda', non_blocking=True)
            dmeta = meta.to('cuda', non_blocking=True)
            done = torch.cuda.Event()
            done.record()
        return dblob, dmeta, done, blob, meta

    def _decoded(self, starts):
        """Decoded batches in order, the next ones already in flight."""
        if self.procs is not None:
            inflight = [self._submit_procs(s) for s in starts[:self.depth]]
            for k in range(len(starts)):
                chunks = inflight.pop(0).get()
                if k + self.depth < len(starts):
                    inflight.append(self._submit_procs(starts[k + self.depth]))
                yield [im for c in chunks for im in c]
            return
        pending = self.pool.submit(self._decode_batch, starts[0]) if starts else None
        for k in range(len(starts)):
            ims = pending.result()
            if k + 1 < len(starts):
                pending = self.pool.submit(self._decode_batch, starts[k + 1])
            yield ims

    def __iter__(self):
        starts = list(range(0, self.n, self.batch))
        for s, ims in zip(starts, self._decoded(starts)):
            dblob, dmeta, done, _hb, _hm = self._stage(ims)
            torch.cuda.current_stream().wait_event(done)
            offs = dmeta[0].contiguous()
            hs = dmeta[1].to(torch.int32).contiguous()
            ws = dmeta[2].to(torch.int32).contiguous()
            x = ops.preprocess_bgr_ragged(dblob, offs, hs, ws, self.means, (self.H, self.W))
            # both staged buffers were allocated on copy_stream and are read
            # on this stream: keep the allocator from recycling either block
            # for the next batch's copy before the kernel above has run
            dblob.record_stream(torch.cuda.current_stream())
            dmeta.record_stream(torch.cuda.current_stream())
            yield s, x


def extract_features(model, source, n, batch=None, out=None, workers=8, paths=None):
    """Features [n, D] (device tensor) for images source(0..n-1): decoded by
    the decode processes when `paths` is given and decode_pool.start() ran,
    else on `workers` host threads."""
    batch = batch or int(cfg.TEST.get('IMS_PER_BATCH', 64))
    feats = out if out is not None else torch.empty((n, model.feat_dim),
                                                    dtype=torch.float32, device='cuda')
    for s, x in BatchFeeder(source, n, batch, workers=workers, paths=paths):
        model.forward(x, out=feats[s:s + x.shape[0]])
    return feats


def get_roidb_and_dataset(dataset_name, ind_range):
    """test_engine.py:408-425 (sorted roidb, optional [start, end) range)."""
    dataset = JsonDataset(dataset_name)
    roidb = dataset.get_roidb(gt=True)
    if ind_range is not None:
        start, end = ind_range
        roidb = roidb[start:end]
    else:
        start, end = 0, len(roidb)
    return roidb, dataset, start, end, len(roidb)


def test_net(weights_file, dataset_name, proposal_file, output_dir, ind_range=None,
             gpu_id=0, model=None, trusted=False):
    """test_engine.py:259-370: features of every image in the (range of the)
    dataset, [N, 3968] float32 on the host; also written to output_dir as
    features.pkl (feature_range_<s>_<e>.pkl for a range) = {'all_feats',
    'cfg'} like the reference's save_object (:356-368)."""
    roidb, dataset, start, end, total = get_roidb_and_dataset(dataset_name, ind_range)
    if model is None:
        model = initialize_model_from_cfg(weights_file, gpu_id, trusted=trusted)
    paths = [e['image'] for e in roidb]
    t0 = time.time()
    feats = extract_features(model, lambda i: _decode_bgr(paths[i]), len(paths), paths=paths)
    torch.cuda.synchronize()
    logger.info('im_detect: %d images in %.2fs (%.1f img/s)', len(paths),
                time.time() - t0, len(paths) / max(time.time() - t0, 1e-9))
    all_feats = feats.cpu().numpy()
    name = 'features.pkl' if ind_range is None else 'feature_range_%s_%s.pkl' % (start, end)
    save_object(dict(all_feats=all_feats, cfg=cfg_yaml()), os.path.join(output_dir, name))
    logger.info('Wrote features to: %s', os.path.abspath(os.path.join(output_dir, name)))
    return all_feats


def cfg_yaml():
    """envu.yaml_dump(cfg) (utils/env.py): the config as a YAML string."""
    import yaml

    def plain(x):
        if isinstance(x, dict):
            return {k: plain(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return [plain(v) for v in x]
        if isinstance(x, np.ndarray):
            return x.tolist()
        return x
    return yaml.safe_dump(plain(cfg))


def save_object(obj, file_name, pickle_format=2):
    """utils/io.py:39-60 save_object: pickle protocol 2 (readable by the
    reference's Python 2 tools), written to a temporary name on the same
    filesystem and renamed into place."""
    import pickle
    import uuid
    file_name = os.path.abspath(file_name)
    tmp = file_name + '.tmp.' + uuid.uuid4().hex
    try:
        with open(tmp, 'wb') as f:
            pickle.dump(obj, f, pickle_format)
        os.rename(tmp, file_name)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def _split_qg(roidb):
    info = [rde.get_info(e) for e in roidb]
    ids = np.array([i[0] for i in info])
    cams = np.array([i[1] for i in info])
    marks = np.array([i[3] for i in info])
    return ids, cams, marks


def multi_gpu_test_net_on_dataset(weights_file, dataset_name, output_dir, trusted=False,
                                  model=None):
    """test_engine.py:184-229 with one process per GPU (already launched by
    torch.distributed.run) instead of subprocesses + pickle files.  Queries,
    gallery and multi-queries are split separately into contiguous shards
    (np.array_split, subprocess.py:53); every rank extracts its shards, the
    features are written once as features.npy (the reference's multi-GPU
    output, :216-227) and the gallery-sharded evaluator computes the same
    (mAP, cmc, mq_mAP, mq_cmc) as the one-GPU evaluate(),
    including multi-query pooling and REID.RERANK (gathered to rank 0).
    Returns the results dict on every rank."""
    rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
    local = int(os.environ.get('LOCAL_RANK', rank))
    roidb, dataset, _, _, _ = get_roidb_and_dataset(dataset_name, None)
    ids, cams, marks = _split_qg(roidb)
    if model is None:
        model = initialize_model_from_cfg(weights_file, local, trusted=trusted)
    paths = [e['image'] for e in roidb]
    shards, rows_of = [], []
    for m in (0, 1, 2):
        rows = np.nonzero(marks == m)[0]
        a, b = pdist.shard_range(len(rows), rank, world)
        sp = [paths[i] for i in rows[a:b]]
        shards.append(extract_features(model, lambda i, sp=sp: _decode_bgr(sp[i]), len(sp),
                                       paths=sp))
        rows_of.append(rows)
    # features in dataset order, written by rank 0 (test_engine.py:216-227):
    # gathered to rank 0 only
    full = None
    for m in (0, 1, 2):
        n = len(rows_of[m])
        if n == 0:
            continue
        sizes = [b - a for a, b in (pdist.shard_range(n, r, world) for r in range(world))]
        allm = pdist.gather_blocks(shards[m], sizes)
        if rank == 0:
            if full is None:
                full = torch.empty((len(paths), model.feat_dim), dtype=torch.float32,
                                   device='cuda')
            full[torch.from_numpy(rows_of[m]).cuda()] = allm
    if rank == 0 and full is not None:
        np.save(os.path.join(output_dir, 'features.npy'), full.cpu().numpy())
    del full
    s = pdist.evaluate_sharded(shards[0], shards[1], shards[2], ids, cams, marks, rank,
                               world, metric=cfg.REID.get('DISTANCE', 'euclidean'),
                               rerank=bool(cfg.REID.RERANK))
    if rank == 0:
        print('{:<30}'.format('Single Query:'), end='')
        rde.print_scores(s[0], s[1])
        if s[2] is not None:
            print('{:<30}'.format('Multi Query:'), end='')
            rde.print_scores(s[2], s[3])
    return _reid_results(dataset.name, s)


def _reid_results(name, s):
    """task_evaluation.py:345-359."""
    r = OrderedDict([('mAP', -1), ('CMC1', -1), ('CMC5', -1), ('CMC10', -1),
                     ('mq_mAP', -1), ('mq_CMC1', -1), ('mq_CMC5', -1), ('mq_CMC10', -1)])
    r['mAP'], r['CMC1'], r['CMC5'], r['CMC10'] = s[0], s[1][0], s[1][4], s[1][9]
    if s[2] is not None:
        r['mq_mAP'] = s[2]
    if s[3] is not None:
        r['mq_CMC1'], r['mq_CMC5'], r['mq_CMC10'] = s[3][0], s[3][4], s[3][9]
    return OrderedDict([(name, OrderedDict(ReID=r))])


def evaluate_reid(dataset, all_feats, output_dir):
    """task_evaluation.py:54-60."""
    s = rde.evaluate(dataset, all_feats, output_dir)
    return _reid_results(dataset.name, s)


def test_net_on_dataset(weights_file, dataset_name, proposal_file, output_dir,
                        multi_gpu=False, gpu_id=0, trusted=False):
    """test_engine.py:146-181."""
    if multi_gpu and torch.distributed.is_initialized() and \
            torch.distributed.get_world_size() > 1:
        return multi_gpu_test_net_on_dataset(weights_file, dataset_name, output_dir,
                                             trusted=trusted)
    dataset = JsonDataset(dataset_name)
    t0 = time.time()
    all_feats = test_net(weights_file, dataset_name, proposal_file, output_dir,
                         gpu_id=gpu_id, trusted=trusted)
    logger.info('Total inference time: {:.3f}s'.format(time.time() - t0))
    return evaluate_reid(dataset, all_feats, output_dir)


def run_inference(weights_file, ind_range=None, multi_gpu_testing=False, gpu_id=0,
                  check_expected_results=False, trusted=False):
    """test_engine.py:91-143."""
    if ind_range is not None:  # child case: features of one range only
        name = cfg.TEST.DATASETS[0]
        return test_net(weights_file, name, None, get_output_dir(name), ind_range=ind_range,
                        gpu_id=gpu_id, trusted=trusted)
    all_results = OrderedDict()
    for name in cfg.TEST.DATASETS:
        all_results.update(test_net_on_dataset(weights_file, name, None,
                                               get_output_dir(name),
                                               multi_gpu=multi_gpu_testing,
                                               gpu_id=gpu_id, trusted=trusted))
    return all_results
