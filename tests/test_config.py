"""Config API parity with the reference's fvcore/yacs-based experiment_manager (CPU only)."""
import argparse
from pathlib import Path

import pytest
import torch

from multimodal_siamese_cd_amd.utils import experiment_manager as em
from multimodal_siamese_cd_amd.utils import parsers


def test_base_chain_and_literal_eval_of_strings():
    cfg = em.load_cfg('siamese_mmcr_alpha0500')  # -> siamese_mmcr_base.yaml -> base.yaml
    assert cfg.MODEL.TYPE == 'whatevernet'
    assert cfg.CONSISTENCY_TRAINER.LOSS_FACTOR == 0.5
    assert cfg.TRAINER.BATCH_SIZE == 4
    assert isinstance(cfg.TRAINER.LR, float) and cfg.TRAINER.LR == 1e-4  # '1e-4' is a string for PyYAML
    assert cfg.NAME == 'siamese_mmcr_alpha0500'
    assert list(cfg.MODEL.TOPOLOGY) == [64, 128, 256, 512]


def test_baseline_configs_exist():
    for name in ('debug', 'baseline_siamese', 'baseline_dualstream', 'dtsiamese', 'siamese_mmcr_alpha0500'):
        cfg = em.load_cfg(name)
        assert cfg.MODEL.TYPE in ('siameseunet', 'dualstreamunet', 'dtsiameseunet', 'whatevernet')
    assert em.load_cfg('baseline_siamese').TRAINER.BATCH_SIZE == 32


def test_merge_from_list_decodes_and_coerces():
    cfg = em.load_cfg('baseline_siamese')
    cfg.merge_from_list(['TRAINER.LR', '3e-4', 'MODEL.TOPOLOGY', '[8, 16]', 'TRAINER.BATCH_SIZE', '2',
                         'NEW.KEY', 'hello'])
    assert cfg.TRAINER.LR == 3e-4 and cfg.MODEL.TOPOLOGY == [8, 16] and cfg.TRAINER.BATCH_SIZE == 2
    assert cfg.NEW.KEY == 'hello'
    with pytest.raises(ValueError):
        cfg.merge_from_list(['TRAINER.LR'])


def test_clone_freeze_dump():
    cfg = em.load_cfg('debug')
    c2 = cfg.clone()
    c2.MODEL.TYPE = 'unet'
    assert cfg.MODEL.TYPE == 'siameseunet'
    cfg.freeze()
    with pytest.raises(AttributeError):
        cfg.MODEL.TYPE = 'x'
    assert 'siameseunet' in cfg.dump()


def test_setup_cfg_with_reference_cli(tmp_path: Path):
    args = parsers.training_argument_parser().parse_args(
        ['-c', 'debug', '-p', 'proj', '-o', str(tmp_path), '-d', str(tmp_path), 'TRAINER.EPOCHS', '3'])
    cfg = em.setup_cfg(args)
    assert cfg.TRAINER.EPOCHS == 3 and cfg.PATHS.OUTPUT == str(tmp_path) and cfg.NAME == 'debug'


def test_relative_base_resolution(tmp_path: Path):
    (tmp_path / 'sub').mkdir()
    (tmp_path / 'a.yaml').write_text("X: 1\nM:\n  A: 1\n  B: '2e-3'\n")
    (tmp_path / 'sub' / 'b.yaml').write_text("_BASE_: '../a.yaml'\nM:\n  A: 5\n")
    cfg = em.new_config()
    cfg.merge_from_file(str(tmp_path / 'sub' / 'b.yaml'))
    assert cfg.X == 1 and cfg.M.A == 5 and cfg.M.B == 2e-3


def test_network_surface_on_cpu_is_parameter_identical_to_reference():
    """Class names / attribute paths / shapes / default init: state_dict keys and shapes as the reference's."""
    import torch
    from multimodal_siamese_cd_amd.utils import networks
    from oracle import siamese_oracle as O
    from oracle.golden import Fixture
    fx = Fixture('dtsiamese_t8-16')
    net = networks.create_network(fx.package_cfg())
    got = [(k, tuple(p.shape)) for k, p in net.module.named_parameters()]
    assert got == list(O.param_shapes(fx.model_type, fx.cfg).items())
    assert all(k.startswith('module.') for k in net.state_dict())
    with pytest.raises(Exception, match='Unknown network'):
        c = fx.package_cfg()
        c.MODEL.TYPE = 'nope'
        networks.create_network(c)
    # the HIP path refuses CPU tensors instead of silently falling back
    x = torch.zeros(1, 5, 32, 32)
    with pytest.raises(RuntimeError):
        net(x, x)


def test_criterion_registry():
    from multimodal_siamese_cd_amd.utils import loss_functions
    assert loss_functions.get_criterion('PowerJaccardLoss') is loss_functions.power_jaccard_loss
    with pytest.raises(NotImplementedError):
        loss_functions.get_criterion('SoftDiceLoss')
    with pytest.raises(Exception, match='unknown loss'):
        loss_functions.get_criterion('Nope')


def test_synthetic_mode_follows_the_split():
    """SYNTHETIC unset: synthetic pairs only when no training AOIs are named (a reference config
    carrying its split must not silently train on noise); an explicit True beside a split warns."""
    import warnings
    from multimodal_siamese_cd_amd.utils import datasets
    cfg = em.load_cfg('baseline_siamese')
    assert cfg.DATALOADER.SYNTHETIC is None and datasets.uses_synthetic_data(cfg)
    cfg.DATASET.TRAINING_IDS = ['L15-0331E-1257N_1327_3160_13']
    assert not datasets.uses_synthetic_data(cfg)
    cfg.DATALOADER.SYNTHETIC = True
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        assert datasets.uses_synthetic_data(cfg)
    assert any('synthetic noise' in str(x.message) for x in w)
    cfg.DATALOADER.SYNTHETIC = False
    cfg.DATASET.TRAINING_IDS = []
    assert not datasets.uses_synthetic_data(cfg)


@pytest.mark.parametrize('config,math', [('baseline_siamese', 'h2'), ('baseline_dualstream', 'bf16'), ('dtsiamese', 'h2'),
                                         ('siamese_mmcr_alpha0500', 'bf16'), ('debug', 'h2')])
def test_create_network_takes_the_arithmetic_from_the_config(config, math):
    """MODEL.PRECISION fp32 -> h2, bf16 -> bf16; MODEL.CONV_MATH overrides; the model carries it (no process mode)."""
    from multimodal_siamese_cd_amd import hip
    from multimodal_siamese_cd_amd.utils import networks
    cfg = em.load_cfg(config)
    assert networks.create_network(cfg).module.conv_math == math
    cfg.MODEL.CONV_MATH = 'x3'
    assert networks.create_network(cfg).module.conv_math == 'x3'
    with hip.conv_scope('f32'):
        assert hip.conv_math() == 'f32'
        with hip.conv_scope(tune=hip.TUNE_WGRAD_R64):
            assert hip.conv_math() == 'f32' and hip.conv_tune() == hip.TUNE_WGRAD_R64
    cfg.MODEL.CONV_MATH = None
    cfg.MODEL.PRECISION = 'fp16'
    with pytest.raises(ValueError, match='PRECISION'):
        networks.create_network(cfg)


def test_topology_and_head_generality_on_cpu():
    """Any topology and any OUT_CHANNELS build with the reference's parameter shapes (the 1x1 head runs in groups of
    4 outputs; channel counts off the granule of 8 run on a padded twin)."""
    from multimodal_siamese_cd_amd.utils import networks
    cfg = em.load_cfg('debug')
    cfg.MODEL.TOPOLOGY = [24, 40]
    cfg.MODEL.OUT_CHANNELS = 7
    net = networks.create_network(cfg)
    assert net.module.outc.conv.weight.shape == (7, 24, 1, 1)
    assert net.module._twin_topo is None


@pytest.mark.parametrize('mtype,topo', [('siameseunet', [12, 20]), ('dualstreamunet', [6, 12]),
                                        ('whatevernet', [5, 9, 14]), ('dtsiameseunet', [3, 7])])
def test_padded_twin_maps_on_cpu(mtype, topo):
    """A topology off the granule of 8: the model keeps the reference's shapes; its twin runs at multiples of 8 and
    every real parameter lands in it at the right positions -- a prefix, or two padded halves for the concat inputs
    (Up's DoubleConv, the fusion heads) -- with zeros elsewhere, and comes back unchanged."""
    from multimodal_siamese_cd_amd.utils import networks
    from oracle import siamese_oracle as O
    cfg = em.load_cfg('debug')
    cfg.MODEL.TYPE, cfg.MODEL.TOPOLOGY = mtype, topo
    net = networks.create_network(cfg).module
    ocfg = dict(TOPOLOGY=topo, IN_CHANNELS=cfg.MODEL.IN_CHANNELS, OUT_CHANNELS=cfg.MODEL.OUT_CHANNELS,
                S1_BANDS=list(cfg.DATALOADER.S1_BANDS), S2_BANDS=list(cfg.DATALOADER.S2_BANDS))
    assert [(k, tuple(p.shape)) for k, p in net.named_parameters()] == list(O.param_shapes(mtype, ocfg).items())
    assert net._twin_topo == [(t + 7) // 8 * 8 for t in topo]
    tw, (maps, bufs) = net._twin_ready('cpu')
    assert list(tw.cfg.MODEL.TOPOLOGY) == net._twin_topo
    for k, p in net.named_parameters():
        shape, m = maps[k]
        big = networks._scatter(p.detach(), shape, m)
        assert tuple(big.shape) == shape
        assert torch.equal(networks._gather(big, m), p.detach())
        assert int((big != 0).sum()) == int((p.detach() != 0).sum())  # zeros everywhere else
        if networks._concat_input(mtype, k):  # two halves: real channel h / 2 sits at padded shape / 2
            h = p.shape[1] // 2
            assert torch.equal(networks._gather(big, [m[0]])[:, shape[1] // 2], p.detach()[:, h])
    for k, b in net.named_buffers():
        assert k in bufs


def test_bf16_storage_needs_every_level_tiled():
    """bf16 storage runs only where every level's map (the input and one per Down: len(TOPOLOGY) + 1 levels) is
    tiled by the bf16 kernels, the deepest a multiple of 16 both ways; other tiles (e.g. full-AOI evaluation) run
    fp32.  The models ask with len(TOPOLOGY) + 1 levels."""
    from multimodal_siamese_cd_amd import engine
    bf, f32 = torch.bfloat16, torch.float32
    assert engine.storage_for_input(bf, 256, 256, 5) == bf  # [64, 128, 256, 512]: deepest 16 x 16
    assert engine.storage_for_input(bf, 128, 128, 5) == f32  # deepest 8 x 8: not tiled
    assert engine.storage_for_input(bf, 128, 128, 4) == bf
    assert engine.storage_for_input(bf, 256, 240, 5) == f32
    assert engine.storage_for_input(f32, 256, 256, 5) == f32
    src = Path(__file__).resolve().parents[1] / 'multimodal_siamese_cd_amd' / 'utils' / 'networks.py'
    assert 'len(self.cfg.MODEL.TOPOLOGY) + 1' in src.read_text()


def test_bf16_storage_needs_a_tiled_input_width():
    """bf16 storage also needs every input layer's padded width (16 or a multiple of 64: the bf16 c16 and
    halo16 kernels); a bf16 config whose padded input has 17-63 channels (e.g. dualstream with 10 S2 bands -> 20 -> 32)
    stores fp32 instead of failing in the input layer's kernels, and an explicit ACT_STORAGE bf16 is refused."""
    from multimodal_siamese_cd_amd import engine
    cfg = em.load_cfg('baseline_dualstream')
    assert engine.input_widths(cfg) == [16, 16]
    assert engine.act_storage_for(cfg) == torch.bfloat16
    cfg.DATALOADER.S2_BANDS = list(range(10))
    assert engine.input_widths(cfg) == [16, 32]
    assert engine.act_storage_for(cfg) == torch.float32
    cfg.MODEL.ACT_STORAGE = 'bf16'
    with pytest.raises(ValueError, match='input widths'):
        engine.act_storage_for(cfg)
    cfg = em.load_cfg('baseline_siamese')
    cfg.MODEL.PRECISION = 'bf16'
    assert engine.input_widths(cfg) == [16] and engine.act_storage_for(cfg) == torch.bfloat16
    cfg.MODEL.IN_CHANNELS = 40  # padded to 48
    assert engine.act_storage_for(cfg) == torch.float32
    cfg.MODEL.IN_CHANNELS = 64
    assert engine.act_storage_for(cfg) == torch.bfloat16
