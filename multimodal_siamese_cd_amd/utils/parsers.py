"""Command-line surface of the training and preprocessing entry points.

Flag-for-flag compatible with the reference's `utils/parsers.py:5-31`: the same short and long options, the same
`dest` names, all required, and a trailing REMAINDER list `opts` of `KEY VALUE` config overrides that
`experiment_manager.setup_cfg` merges (`experiment_manager.py:62`).  Built from one table so the two parsers
cannot drift apart.
"""
import argparse

# (short, long, dest, help) — every option is required, as in the reference
_TRAINING_FLAGS = (
    ('-c', '--config-file', 'config_file', 'config name or path (configs/<name>.yaml)'),
    ('-p', '--project', 'project', 'experiment-tracking project name (wandb in the reference; logged only)'),
    ('-o', '--output-dir', 'output_dir', 'directory for checkpoints and logs'),
    ('-d', '--dataset-dir', 'dataset_dir', 'tile-cache root; synthetic pairs when the config names no AOIs'),
)
_PREPROCESS_FLAGS = (
    ('-d', '--dataset', 'dataset', 'dataset root'),
)


def _build(flags) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description='Experiment Args')
    for short, long_, dest, text in flags:
        p.add_argument(short, long_, dest=dest, required=True, help=text)
    p.add_argument('opts', nargs=argparse.REMAINDER, default=None,
                   help='trailing KEY VALUE pairs that override the config')
    return p


def training_argument_parser() -> argparse.ArgumentParser:
    """`-c/-p/-o/-d` + opts (reference `parsers.py:5-19`)."""
    return _build(_TRAINING_FLAGS)


def preprocess_argument_parser() -> argparse.ArgumentParser:
    """`-d` + opts (reference `parsers.py:22-31`)."""
    return _build(_PREPROCESS_FLAGS)
