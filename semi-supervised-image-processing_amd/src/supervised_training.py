"""CLI wrapper for supervised (baseline) training (drop-in for the
reference's src/supervised_training.py:23-121).

Usage:
    python -m src.supervised_training --strong-data-dir <path>
"""
from __future__ import annotations

import json
import logging
from typing import Optional, Sequence

from training.common import TrainingConfig
from training.supervised import run_supervised

from ._cli import base_parser, to_config

LOGGER = logging.getLogger(__name__)


def parse_args(args: Optional[Sequence[str]] = None) -> TrainingConfig:
    return to_config(base_parser(__doc__, weak_required=False).parse_args(args=args), semi=False)


def main(args: Optional[Sequence[str]] = None) -> None:
    logging.basicConfig(level=logging.INFO, format="[%(asctime)s] %(levelname)s:%(name)s:%(message)s")
    config = parse_args(args)
    metrics = run_supervised(config)
    LOGGER.info("Baseline training complete. Metrics:\n%s", json.dumps(metrics, indent=2))


if __name__ == "__main__":  # pragma: no cover
    main()
