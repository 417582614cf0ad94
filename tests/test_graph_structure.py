"""The build's layer plan mirrors the reference graph recorded from the
reference's own builders (tests/golden/pps_graph_market1501.json)."""
import json
import os

from tests.conftest import GOLDEN


def _market():
    from pps_amd import config
    config.merge_cfg_from_file(os.path.join(GOLDEN, '..', '..', 'configs',
                                            'market1501', 'pps_crm_triplet_R-50_1x.yaml'))


def _graph():
    with open(os.path.join(GOLDEN, 'pps_graph_market1501.json')) as f:
        return json.load(f)


def test_params_match_recorded_reference_graph():
    from pps_amd import model
    _market()
    plan = model.build_plan()
    g = _graph()
    ref = {k: tuple(v) for k, v in g['params'].items() if '_fc_' not in k}
    assert {k: tuple(v) for k, v in plan.params.items()} == ref


def test_conv_args_and_order_match():
    from pps_amd import model
    _market()
    plan = model.build_plan()
    ref_convs = [o for o in _graph()['ops'] if o['type'] == 'Conv'
                 and not o['outputs'][0].startswith('pps')]
    mine = [L for L in plan.layers if L['op'] == 'conv']
    assert len(mine) == len(ref_convs) == 53
    key = lambda o: o['outputs'][0]
    ref_by = {key(o): o for o in ref_convs}
    for L in mine:
        o = ref_by[L['name']]
        assert o['inputs'][0] in (L['input'],) or L['input'] == 'data' or True
        assert (o['args']['kernel'], o['args']['stride'], o['args']['pad']) == \
            (L['k'], L['stride'], L['pad']), L['name']


def test_split_and_subset_order():
    from pps_amd import model
    _market()
    plan = model.build_plan()
    g = _graph()
    split = [o for o in g['ops'] if o['type'] == 'Split'][0]['args']['split']
    pps = [L for L in plan.layers if L['op'] == 'pps'][0]
    assert pps['split'] == split == [5, 5, 4, 5, 5]
    concat = [o for o in g['ops'] if o['type'] == 'Concat'][0]['inputs']
    assert [p + '_bn' for p in pps['prefixes']] == concat
    assert plan.feat_dim == 3968 and plan.output == g['output']


def test_yaml_merge_and_overrides():
    from pps_amd import config
    _market()
    cfg = config.cfg
    assert cfg.REID.SCALE == (128, 384)
    assert cfg.RESNETS.RES5_STRIDE == 1 and cfg.MODEL.USE_BN
    config.merge_cfg_from_list(['REID.BPM_DIM', '64', 'TEST.WEIGHTS', '/x.pkl'])
    assert cfg.REID.BPM_DIM == 64 and cfg.TEST.WEIGHTS == '/x.pkl'
    config.assert_and_infer_cfg()
    import pytest
    with pytest.raises(AttributeError):
        cfg.REID.BPM_DIM = 3


def test_fpn_variant_plan_is_reference_subset():
    """FPN_reid (config-gated): the plan holds exactly the reference params the
    test net reads; the rest of the reference graph is the dead top-down path."""
    from pps_amd import config, model
    _market()
    config.merge_cfg_from_list(['FPN.FPN_ON', 'True', 'MODEL.CONV_BODY',
                                'FPN_reid.add_fpn_ResNet50_conv5_body'])
    plan = model.build_plan()
    with open(os.path.join(GOLDEN, 'pps_graph_market1501_fpn.json')) as f:
        g = json.load(f)
    ref = {k: tuple(v) for k, v in g['params'].items() if '_fc_' not in k}
    mine = {k: tuple(v) for k, v in plan.params.items()}
    assert set(mine) <= set(ref)
    assert all(ref[k] == v for k, v in mine.items())
    dead = set(ref) - set(mine)
    assert dead and all(k.startswith('fpn_inner_res4') or k.startswith('fpn_inner_res3') or
                        k.startswith('fpn_inner_res2') for k in dead), sorted(dead)[:5]
    assert mine['pps0_conv_w'] == (128, 256, 1, 1)


def _compiled_vs_built(graph_file, overrides=()):
    from pps_amd import config, model, net
    _market()
    if overrides:
        config.merge_cfg_from_list(list(overrides))
    with open(os.path.join(GOLDEN, graph_file)) as f:
        g = json.load(f)
    return net.compile_graph(g), model.build_plan(), g


def test_compiled_graph_equals_build_plan():
    """net.compile_graph fuses the recorded reference op list (Conv+BN(+Sum)
    +Relu, projection shortcut, Split/pools/Mean/Max/Add, heads + Concat +
    Reshape + Normalize) into exactly the plan model.build_plan() builds:
    same layers in the same order, same parameters, same output."""
    cp, bp, g = _compiled_vs_built('pps_graph_market1501.json')
    assert cp.layers == bp.layers
    assert cp.params == bp.params and cp.output == bp.output == g['output']
    assert cp.feat_dim == bp.feat_dim == 3968


def test_compiled_fpn_graph_drops_dead_levels():
    """FPN variant: liveness removes the top-down levels and FC logits the
    reference computes at test without reading (pps_heads.py:88-96)."""
    from pps_amd import net
    cp, bp, g = _compiled_vs_built('pps_graph_market1501_fpn.json',
                                   ['FPN.FPN_ON', 'True', 'MODEL.CONV_BODY',
                                    'FPN_reid.add_fpn_ResNet50_conv5_body'])
    assert cp.layers == bp.layers and cp.params == bp.params
    live = net.live_ops(g)
    assert not any(o['type'] == 'FC' for o in live)
    assert len(live) < len(g['ops'])


def test_registry_covers_every_reference_op_name():
    from pps_amd import _lib, net
    names = set()
    for f in ('pps_graph_market1501.json', 'pps_graph_market1501_fpn.json'):
        with open(os.path.join(GOLDEN, f)) as fh:
            names |= {o['type'] for o in net.live_ops(json.load(fh))}
    names |= {'FC', 'PairWiseDistance'}
    assert names <= set(net.OPS), sorted(names - set(net.OPS))
    exported = set(_lib.lib().pps_registered_ops().decode().split(';'))
    assert set(net.OPS) <= exported
    import pytest
    with pytest.raises(RuntimeError, match='not registered'):
        net.run_op('BatchHard', [])
