"""The f16x2 layers in the whole-network plan (PPS_TILE_H2, include/pps_abi.h):

* every producer reports max|y| of its output in the forward (x3 pipelined,
  patch, weight-stationary and register-staged tiles, the bottleneck seam,
  the fused stem and the unfused max pooling): the slot equals max|t| of the
  tensor exactly -- these are the f16x2 layers' input scales;
* a table with PPS_TILE_H2 layers (every base tile family) runs the same
  bits in the C plan and in the Python orchestrator (which measures its
  inputs' maxima with pps_amax), also under hipGraph replay, and stays
  within FWD_ATOL of the CPU oracle;
* PPS_TILE_H2E edges (the producer writes f16x2 planes on the scale of its
  output bound, bf16x3 or f16x2 producers): C plan == twin bit for bit,
  within FWD_ATOL of the oracle, under graph replay; the planes decode to the
  producer's f32 output within 2^-21 of the bound;
* the C autotune with f16x2 candidates gives a table the Python orchestrator
  reproduces bit for bit;
* the plan refuses PPS_TILE_H2 where it cannot run."""
import numpy as np
import pytest
import torch

from tests.test_gpu_native import FWD_ATOL, _input, _models

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('variant', ['default', 'mixed_tiles', 'unfused_stem'])
def test_producers_report_tensor_max(variant, monkeypatch):
    from pps_amd import ops
    monkeypatch.setenv('PPS_AMAX_ALL', '1')   # all producers, not only those h2 layers read
    kw = dict(fused_stem=False) if variant == 'unfused_stem' else {}
    _, pm, nm = _models(seed=3, **kw)
    N = 2
    _, x = _input(N, seed=4)
    if variant == 'mixed_tiles':
        # register-staged, pipelined 32x32 / 16x16, weight-stationary, patch
        # and a seam pair -- every epilogue family reports its maximum
        fam = [1, 11, 22, 30, 36, 40, 47, 52, 54, 56]
        t = {}
        for i, L in enumerate(nm.layers(N)):
            if L['op'] in ('conv', 'conv_dual'):
                t[L['name']] = fam[i % len(fam)]
        t['res2_1_branch2c'] = 54 | ops.TILE_SEAM
        nm.set_planes([])
        nm.set_tiles(t)
    nm.forward(x)
    checked = skipped = 0
    for L in nm.layers(N):
        if L['op'] not in ('conv', 'conv_dual', 'maxpool', 'stem_pool'):
            continue
        if L['planes_out']:   # a bf16x3 plane edge: no f32 tensor to measure
            skipped += 1
            continue
        t = nm.tensor(N, L['output'])
        got = nm.tensor_amax(N, L['output'])
        assert got == float(np.abs(t).max()), (L['output'], got, float(np.abs(t).max()))
        checked += 1
    # the architecture's f32 producers: 16 bottlenecks x 3 convs, less the
    # last branch2c (the fused part pooling), + the stem (one fused launch,
    # or conv1 + pool1); every one is checked unless it writes plane edges
    n_arch = 47 + (2 if variant == 'unfused_stem' else 1)
    assert checked + skipped == n_arch, (checked, skipped)
    assert skipped == len(nm.planes()), (skipped, nm.planes())


def _h2_table(nm, N):
    """Every f16x2-capable layer on an f16x2 tile, cycling the base families
    (_apply puts the weight-stationary 1x1s on tile 54)."""
    from pps_amd import ops
    fam = [0, 38, 43, 47, 50, 52, 55, 56, 59]
    t = {}
    k = 0
    for L in nm.layers(N):
        if L['op'] in ('conv', 'conv_dual', 'conv_pps', 'stem_pool'):
            t[L['name']] = L['tile']
    for name in list(t):
        L = next(M for M in nm.layers(N) if M['name'] == name)
        if L['op'] == 'stem_pool':   # the fused stem: its own kernel, f16x2 or not
            t[name] = ops.TILE_H2
            continue
        base = fam[k % len(fam)]
        k += 1
        if L['op'] == 'conv_dual' and base >= 56:
            base = 47
        if L['op'] == 'conv_pps':
            base = 47
        t[name] = base | ops.TILE_H2
        if L['op'] != 'conv_dual' and k % 2:   # every other one on split-once input planes
            t[name] |= ops.TILE_H2P
    return t


def _apply(nm, table):
    """Set each layer's tile of `table` the plan accepts -- the f16x2
    weight-stationary tile 54 first wherever the plan takes it (1x1 / stride
    1 / K = 64, 128, 256: res2 2a / 2c, the res2_0 shortcut conv, res3 2c,
    res4 2c); the accepted table."""
    from pps_amd import ops
    ok = {}
    for name, t in table.items():
        for tt in (ops.TILE_WS | ops.TILE_H2, t):
            try:
                nm.set_tiles({name: tt})
                ok[name] = tt
                break
            except RuntimeError:
                nm.set_tiles({name: 0})
    return ok


def test_h2_table_c_plan_equals_twin_and_oracle():
    from oracle.forward import GraphForward
    from pps_amd import ops
    blobs, pm, nm = _models(seed=5)
    N = 3
    x, xd = _input(N, seed=6)
    nm.set_planes([])
    pm.set_planes([])
    ok = _apply(nm, _h2_table(nm, N))   # the layers the plan accepts (Cin % 32 == 0)
    assert len(ok) >= 45, len(ok)
    assert ok.get('conv1') == ops.TILE_H2, ok.get('conv1')   # the f16x2 fused stem
    assert sum(1 for t in ok.values() if (t & 0xff) == ops.TILE_WS) >= 4   # f16x2 ws 1x1s
    assert sum(1 for t in ok.values() if t & ops.TILE_H2P) >= 12
    pm.set_tiles(ok)
    a = pm.forward(xd).cpu().numpy()
    b = nm.forward(xd).cpu().numpy()
    assert np.array_equal(a, b)
    ref = GraphForward(blobs)(x).numpy()
    err = float(np.abs(b - ref).max())
    print('f16x2 table (%d layers) forward max|err| vs oracle %.3g' % (len(ok), err))
    assert err <= FWD_ATOL
    # graph replay (the amax slots are zeroed by a memset node every replay)
    nm.reserve(N)
    out = torch.empty((N, nm.feat_dim), device='cuda')
    nm.forward(xd, out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nm.forward(xd, out=out)
    out.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), b)


def _h2e_table(nm, pm, N):
    """_h2_table with PPS_TILE_H2E on every consumer the plan accepts; every
    third accepted edge gets a bf16x3 producer (tile 47).  Returns (table, edges)
    with edges = [(producer, consumer)]."""
    from pps_amd import ops
    layers = nm.layers(N)
    ok = _apply(nm, _h2_table(nm, N))
    edges = []
    for L in layers:
        name = L['name']
        if name not in ok or not ok[name] & ops.TILE_H2 or L['op'] not in ('conv', 'conv_pps'):
            continue
        t = (ok[name] & ~ops.TILE_H2P) | ops.TILE_H2E
        try:
            nm.set_tiles({name: t})
        except RuntimeError:
            continue
        ok[name] = t
        C = next(M for M in pm.layers if M.get('name') == name)   # the twin has the inputs
        P = next(M['name'] for M in pm.layers if M['output'] == C['input'])
        if len(edges) % 3 == 0 and not ok.get(P, 0) & ops.TILE_H2E:
            ok[P] = 47
            nm.set_tiles({P: 47})
        edges.append((P, name))
    return ok, edges


def test_h2e_edges_c_plan_equals_twin_and_oracle():
    from oracle.forward import GraphForward
    from pps_amd import ops
    blobs, pm, nm = _models(seed=11)
    N = 3
    x, xd = _input(N, seed=12)
    nm.set_planes([])
    pm.set_planes([])
    ok, edges = _h2e_table(nm, pm, N)
    print('PPS_TILE_H2E edges: %d' % len(edges))
    # (the weight-stationary 2c layers read f32: 14 consumers or more)
    assert len(edges) >= 14, edges
    assert any(not ok[p] & ops.TILE_H2 for p, _ in edges)   # bf16x3 producers too
    # f16x2 weight-stationary producers writing the planes (gemm_ws.hip H2O)
    assert any((ok[p] & 0xff) == ops.TILE_WS and ok[p] & ops.TILE_H2 for p, _ in edges), edges
    pm.set_tiles(ok)
    a = pm.forward(xd).cpu().numpy()
    b = nm.forward(xd).cpu().numpy()
    assert np.array_equal(a, b)
    ref = GraphForward(blobs)(x).numpy()
    err = float(np.abs(b - ref).max())
    print('f16x2 table with planes edges: max|err| vs oracle %.3g' % err)
    assert err <= FWD_ATOL
    # the planes decode to the producer's f32 output (the same table without
    # that edge's flag: everything upstream of the producer is unchanged)
    layers = {L['name']: L for L in nm.layers(N)}
    for p, c in (edges[0], edges[1], edges[-1]):
        if ok[p] & ops.TILE_H2E:
            continue
        blob = layers[p]['output']
        dec = nm.tensor(N, blob)
        bnd = nm.tensor_amax(N, blob)
        nm.set_tiles({c: ok[c] & ~ops.TILE_H2E})
        nm.forward(xd)
        y = nm.tensor(N, blob)
        nm.set_tiles({c: ok[c]})
        assert bnd >= float(np.abs(y).max()) > 0
        d = float(np.abs(dec.astype(np.float64) - y).max())
        assert d <= bnd * 2.0 ** -21, (p, c, d, bnd)
    # graph replay
    nm.forward(xd)
    nm.reserve(N)
    out = torch.empty((N, nm.feat_dim), device='cuda')
    nm.forward(xd, out=out)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nm.forward(xd, out=out)
    out.zero_()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), b)


def test_autotune_with_h2_candidates_then_twin():
    from pps_amd import ops
    _, pm, nm = _models(seed=7)
    _, x = _input(2, seed=8)
    tiles = nm.autotune(x)
    nh2 = sum(1 for t in tiles.values() if t & ops.TILE_H2)
    print('autotune: %d of %d layers on f16x2 tiles' % (nh2, len(tiles)))
    pm.set_tiles(tiles)
    pm.set_planes(nm.planes())
    pm.set_splitks(nm.splitks())
    assert np.array_equal(pm.forward(x).cpu().numpy(), nm.forward(x).cpu().numpy())
    # the flag keeps the bf16x3 table
    tiles2 = nm.autotune(x, flags=8)
    assert not any(t & ops.TILE_H2 for t in tiles2.values())


def test_h2_tile_refused_where_it_cannot_run():
    from pps_amd import ops
    _, pm, nm = _models(seed=9)
    with pytest.raises(RuntimeError, match='PPS_TILE_H2'):
        nm.set_tiles({'reid_feature_concat_norm': 38 | ops.TILE_H2})   # heads
    with pytest.raises(RuntimeError, match='PPS_TILE_H2'):
        nm.set_tiles({'res2_0_branch2b': 30 | ops.TILE_H2})           # a 32x32 tile
    with pytest.raises(ValueError, match='PPS_TILE_H2'):
        pm.set_tiles({'res2_0_branch2b': 30 | ops.TILE_H2})
    dual = next(L['name'] for L in nm.layers() if L['op'] == 'conv_dual')
    with pytest.raises(RuntimeError, match='PPS_TILE_H2P'):
        nm.set_tiles({dual: 47 | ops.TILE_H2 | ops.TILE_H2P})   # the shortcut reads f32
    with pytest.raises(RuntimeError, match='PPS_TILE_H2P'):
        nm.set_tiles({'res2_0_branch2b': 38 | ops.TILE_H2P})     # without PPS_TILE_H2
    with pytest.raises(ValueError, match='PPS_TILE_H2P'):
        pm.set_tiles({dual: 47 | ops.TILE_H2 | ops.TILE_H2P})
    # PPS_TILE_H2E: not on the pool's reader (maxpool producer), not without
    # PPS_TILE_H2, not with PPS_TILE_H2P, not on a conv_dual
    for bad in [('res2_0_branch2a', 38 | ops.TILE_H2 | ops.TILE_H2E),
                ('res2_0_branch2b', 38 | ops.TILE_H2E),
                ('res2_0_branch2b', 38 | ops.TILE_H2 | ops.TILE_H2P | ops.TILE_H2E),
                (dual, 47 | ops.TILE_H2 | ops.TILE_H2E)]:
        with pytest.raises(RuntimeError, match='PPS_TILE_H2'):
            nm.set_tiles(dict([bad]))
        with pytest.raises(ValueError, match='PPS_TILE_H2'):
            pm.set_tiles(dict([bad]))
    nm.set_tiles({'res2_0_branch2b': 38 | ops.TILE_H2 | ops.TILE_H2E})
    pm.set_tiles({'res2_0_branch2b': 38 | ops.TILE_H2 | ops.TILE_H2E})
    # a plane edge into an f16x2 layer is refused, in either order
    edges = nm.plane_edges()
    p, c, _ = edges[0]
    nm.set_planes([])
    nm.set_tiles({c: 38 | ops.TILE_H2})
    with pytest.raises(RuntimeError, match='f16x2'):
        nm.set_planes([p])


def test_h2_features_batch_invariant_within_tolerance():
    """the f16x2 layers scale activations by one power of two per
    tensor, from the max over the whole batch, so an image's features depend
    on its batch-mates at f32-rounding level (the reference runs one image
    per RunNet; DESIGN §2 states this).  The bound that matters: an image
    alone (N = 1) and the same image inside a batch whose other images are
    10x brighter give features within FWD_ATOL of each other, and each within
    FWD_ATOL of the oracle."""
    from oracle.forward import GraphForward
    blobs, pm, nm = _models(seed=13)
    N = 3
    x, _ = _input(N, seed=14)
    x[1:] *= 10.0   # batch-mates with a 10x larger activation range
    xin = np.zeros((N, 384, 128, 4), np.float32)
    xin[..., :3] = x.transpose(0, 2, 3, 1)
    nm.set_planes([])
    _apply(nm, _h2_table(nm, N))
    batch = nm.forward(torch.from_numpy(xin).cuda()).cpu().numpy()
    alone = nm.forward(torch.from_numpy(xin[:1].copy()).cuda()).cpu().numpy()
    ref = GraphForward(blobs)(x[:1]).numpy()
    d = float(np.abs(batch[0] - alone[0]).max())
    print('image 0 alone vs in a 10x-brighter batch: max|diff| %.3g' % d)
    assert d <= FWD_ATOL
    assert float(np.abs(alone - ref).max()) <= FWD_ATOL
    assert float(np.abs(batch[:1] - ref).max()) <= FWD_ATOL


def test_layer_ranges_measure_fresh_maxima():
    """a layer range run after a forward on a LARGER input gives
    the bits of a whole forward on the small input -- the range zeroes the
    maxima slots of the tensors it produces, so no stale, larger scale from
    the earlier call reaches its f16x2 consumers."""
    _, pm, nm = _models(seed=15)
    N = 2
    _, xs = _input(N, seed=16)
    xl = xs * 20.0
    nm.set_planes([])
    _apply(nm, _h2_table(nm, N))
    want = nm.forward(xs).cpu().numpy()
    n = len(nm.layers(N))
    for k in (n // 3, n // 2, n - 3):
        nm.forward(xl)
        out = torch.empty((N, nm.feat_dim), device='cuda')
        nm.forward_layers(xs, 0, k, out=out)
        nm.forward_layers(xs, k, n, out=out)
        assert np.array_equal(out.cpu().numpy(), want), k
