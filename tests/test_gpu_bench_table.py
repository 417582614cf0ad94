"""The configuration bench.py times, built by bench.py's own code
(`build_bench_model`: same seeded weights and images, pps_model_autotune on
THIS device at batch 64 with the bench's flags) -- so the tuning table these
tests check is the one behind `value`, not a committed file from another box
(VERDICT r03 item 4).  Checks: the autotuned C plan equals the Python
orchestrator given the same table bit for bit (also through the uint8 and
NCHW entry points); three of the 64 images' features within FWD_ATOL of the
CPU oracle (the recorded reference graph, oracle/forward.py).  The table's
digest and its layer count per rounding group are printed (bench.py puts the
same digest in its JSON line, config.tuning_table)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FWD_ATOL = 1e-6   # normalised 3968-d features vs the oracle (observed ~6e-8)


@pytest.fixture(scope='module')
def bench_cfg():
    import bench
    from pps_amd import config
    config.reset_cfg()
    nm, blobs, imgs, xbuf = bench.build_bench_model(64, rank=0, autotune=True, flags=0)
    dig = bench.table_digest(nm)
    print('bench table', dig)
    return dict(nm=nm, blobs=blobs, imgs=imgs, x=xbuf, digest=dig)


def test_bench_table_c_plan_equals_python_twin(bench_cfg):
    import bench
    from pps_amd import model
    bench.market_cfg()
    nm, x = bench_cfg['nm'], bench_cfg['x']
    pm = model.PPSModel(bench_cfg['blobs'])
    pm.set_tiles(nm.tiles())
    pm.set_planes(nm.planes())
    pm.set_splitks(nm.splitks())
    assert nm.tiles() == pm.tiles() and sorted(nm.planes()) == sorted(pm.planes())
    a = pm.forward(x).cpu().numpy()
    b = nm.forward(x).cpu().numpy()
    assert np.array_equal(a, b)
    c = nm.forward_bgr(bench_cfg['imgs']).cpu().numpy()
    assert np.array_equal(b, c)
    nchw = x[..., :3].permute(0, 3, 1, 2).contiguous()
    assert np.array_equal(b, nm.forward_nchw(nchw).cpu().numpy())
    # the rounding groups the table uses, as the bench line reports them
    assert sum(bench_cfg['digest']['layers_per_rounding_group'].values()) == len(nm.tiles())


def test_bench_table_vs_oracle(bench_cfg):
    import bench
    from oracle.forward import GraphForward
    bench.market_cfg()
    nm, x = bench_cfg['nm'], bench_cfg['x']
    feat = nm.forward_bgr(bench_cfg['imgs']).cpu().numpy()
    pick = [0, 17, 63]
    # the oracle forward on the kernel's own preprocessed input (preprocess
    # parity is test_gpu_forward.py::test_preprocess_vs_oracle's)
    xin = x[pick, :, :, :3].cpu().numpy().transpose(0, 3, 1, 2)
    ref = GraphForward(bench_cfg['blobs'])(np.ascontiguousarray(xin, np.float32)).numpy()
    err = float(np.abs(feat[pick] - ref).max())
    print('bench table %s: forward max|err| vs oracle %.3g'
          % (bench_cfg['digest']['sha1'], err))
    assert err <= FWD_ATOL
