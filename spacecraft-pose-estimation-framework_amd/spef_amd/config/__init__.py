"""Experiment configuration: the reference's YAML surface (src/config/train/config.py:4-42, yacs ``CfgNode``),
read with ``yaml.safe_load`` (no yacs here), plus the ``MI355X`` section the build/deploy tools add."""
from .config import load_config, save_config, to_spe_utils  # noqa: F401
