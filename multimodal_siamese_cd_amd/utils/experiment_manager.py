"""YAML experiment configuration — drop-in for the reference's utils/experiment_manager.py.

The reference subclasses fvcore's CfgNode (experiment_manager.py:11-35; fvcore is not installed and not
fetchable here), so the semantics it relies on are restated from scratch:

  * attribute access (`cfg.MODEL.TYPE`), nested nodes, new keys always allowed (networks read keys the
    defaults never declare, experiment_manager.py:24-27);
  * `merge_from_file` with `_BASE_` inheritance resolved relative to the including file, recursively
    (e.g. configs/siamese_mmcr_alpha0500.yaml -> siamese_mmcr_base.yaml -> base.yaml);
  * yacs-style value decoding: string values go through ast.literal_eval, so `LR: 1e-4` (a *string* for
    PyYAML) becomes the float 1e-4 (as the reference's trainers rely on, train_supervised.py:32);
  * `merge_from_list(["KEY.SUB", "VALUE", ...])` for CLI overrides (experiment_manager.py:62);
  * `clone()`, `dump()`, `freeze()`/`defrost()`.

YAML is loaded with yaml.safe_load (the reference's unsafe loading is deliberately not reproduced).
"""
from __future__ import annotations

import ast
import copy
from pathlib import Path

import yaml

BASE_KEY = '_BASE_'
_PKG_CONFIGS = Path(__file__).resolve().parent.parent / 'configs'


def _decode(v):
    if isinstance(v, dict):
        return CfgNode(v)
    if isinstance(v, str):
        try:
            return ast.literal_eval(v)
        except (ValueError, SyntaxError):
            return v
    if isinstance(v, list):
        return [_decode(x) if isinstance(x, (dict, str)) else x for x in v]
    return v


class CfgNode(dict):
    IMMUTABLE = '__immutable__'

    def __init__(self, init_dict=None, key_list=None, new_allowed=True):
        super().__init__()
        object.__setattr__(self, CfgNode.IMMUTABLE, False)
        for k, v in (init_dict or {}).items():
            self[k] = _decode(v) if isinstance(v, dict) else v

    # attribute access ---------------------------------------------------------------------------
    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name) from None

    def __setattr__(self, name, value):
        if self.__dict__.get(CfgNode.IMMUTABLE, False):
            raise AttributeError(f'Attempted to set {name} to {value}, but CfgNode is immutable')
        self[name] = value

    def __setitem__(self, key, value):
        if self.__dict__.get(CfgNode.IMMUTABLE, False):
            raise AttributeError(f'Attempted to set {key} to {value}, but CfgNode is immutable')
        if isinstance(value, dict) and not isinstance(value, CfgNode):
            value = CfgNode(value)
        super().__setitem__(key, value)

    # yacs API -----------------------------------------------------------------------------------
    def freeze(self):
        self._set_immutable(True)

    def defrost(self):
        self._set_immutable(False)

    def is_frozen(self):
        return self.__dict__[CfgNode.IMMUTABLE]

    def _set_immutable(self, flag):
        object.__setattr__(self, CfgNode.IMMUTABLE, flag)
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_immutable(flag)

    def clone(self):
        return copy.deepcopy(self)

    def __deepcopy__(self, memo):
        out = CfgNode()
        for k, v in self.items():
            out[k] = copy.deepcopy(v, memo)
        object.__setattr__(out, CfgNode.IMMUTABLE, self.__dict__[CfgNode.IMMUTABLE])
        return out

    def to_dict(self):
        return {k: (v.to_dict() if isinstance(v, CfgNode) else v) for k, v in self.items()}

    def dump(self, **kw):
        return yaml.safe_dump(self.to_dict(), **kw)

    @staticmethod
    def load_yaml_with_base(filename, allow_unsafe: bool = False):
        """Load a YAML file, recursively merging the `_BASE_` chain (paths relative to the file)."""
        filename = Path(filename)
        with open(filename) as f:
            cfg = yaml.safe_load(f) or {}
        base = cfg.pop(BASE_KEY, None)
        if base is None:
            return cfg
        base_path = Path(base).expanduser()
        if not base_path.is_absolute():
            base_path = filename.parent / base_path
        base_cfg = CfgNode.load_yaml_with_base(base_path, allow_unsafe)

        def merge(a, b):  # b into a
            for k, v in b.items():
                if isinstance(v, dict) and isinstance(a.get(k), dict):
                    merge(a[k], v)
                else:
                    a[k] = v
            return a

        return merge(base_cfg, cfg)

    def merge_from_file(self, cfg_filename, allow_unsafe: bool = True):
        loaded = CfgNode.load_yaml_with_base(cfg_filename, allow_unsafe)
        self.merge_from_other_cfg(CfgNode(loaded))

    def merge_from_other_cfg(self, other):
        _merge_into(other, self)

    def merge_from_list(self, cfg_list):
        cfg_list = list(cfg_list or [])
        if len(cfg_list) % 2:
            raise ValueError(f'Override list has odd length: {cfg_list}')
        for full_key, v in zip(cfg_list[0::2], cfg_list[1::2]):
            keys = full_key.split('.')
            d = self
            for sub in keys[:-1]:
                if sub not in d:
                    d[sub] = CfgNode()
                d = d[sub]
            d[keys[-1]] = _coerce(_decode(v), d.get(keys[-1]), full_key)


def _coerce(new, old, key):
    if old is None or new is None or type(new) is type(old):
        return new
    if isinstance(old, float) and isinstance(new, int) and not isinstance(new, bool):
        return float(new)
    if isinstance(old, (list, tuple)) and isinstance(new, (list, tuple)):
        return type(old)(new)
    if isinstance(old, str) and not isinstance(new, str):
        return new
    if isinstance(old, (int, float)) and isinstance(new, (int, float)):
        return new
    raise ValueError(f'Type mismatch ({type(old).__name__} vs {type(new).__name__}) for config key {key}')


def _merge_into(a, b):
    """Recursively merge CfgNode a into b, decoding string values (yacs _merge_a_into_b)."""
    for k, v in a.items():
        v = _decode(v) if not isinstance(v, CfgNode) else v
        if isinstance(v, CfgNode):
            if not isinstance(b.get(k), CfgNode):
                b[k] = CfgNode()
            _merge_into(v, b[k])  # decodes the strings of new subtrees too
        else:
            b[k] = copy.deepcopy(v)


def new_config():
    """experiment_manager.py:38-56."""
    C = CfgNode()
    C.CONFIG_DIR = 'config/'
    C.PATHS = CfgNode()
    C.TRAINER = CfgNode()
    C.MODEL = CfgNode()
    C.DATALOADER = CfgNode()
    C.AUGMENTATIONS = CfgNode()
    C.CONSISTENCY_TRAINER = CfgNode()
    C.DATASETS = CfgNode()
    return C.clone()


def _config_file(name: str) -> Path:
    """configs/<name>.yaml relative to the CWD (reference behaviour, :61), else the packaged configs."""
    p = Path('configs') / f'{name}.yaml'
    if p.exists():
        return p
    q = _PKG_CONFIGS / f'{name}.yaml'
    if q.exists():
        return q
    raise FileNotFoundError(f'config {name}: neither {p} nor {q} exists')


def setup_cfg(args):
    """experiment_manager.py:59-69."""
    cfg = new_config()
    cfg.merge_from_file(str(_config_file(args.config_file)))
    cfg.merge_from_list(args.opts)
    cfg.NAME = args.config_file
    cfg.PATHS.ROOT = str(Path.cwd())
    assert Path(args.output_dir).exists()
    cfg.PATHS.OUTPUT = args.output_dir
    assert Path(args.dataset_dir).exists()
    cfg.PATHS.DATASET = args.dataset_dir
    return cfg


def setup_cfg_manual(config_name: str, output_dir: Path, dataset_dir: Path):
    """experiment_manager.py:72-81."""
    cfg = new_config()
    cfg.merge_from_file(str(_config_file(config_name)))
    cfg.NAME = config_name
    cfg.PATHS.ROOT = str(Path.cwd())
    assert Path(output_dir).exists()
    cfg.PATHS.OUTPUT = str(output_dir)
    assert Path(dataset_dir).exists()
    cfg.PATHS.DATASET = str(dataset_dir)
    return cfg


def load_cfg(config_name: str):
    """experiment_manager.py:85-90."""
    cfg = new_config()
    cfg.merge_from_file(str(_config_file(config_name)))
    cfg.NAME = config_name
    return cfg
