"""Semi-supervised training CLI (drop-in for the reference's
src/semi_supervised_training.py:521-650).

Usage:
    python -m src.semi_supervised_training --strong-data-dir <labelled> --weak-data-dir <unlabelled>
"""
from __future__ import annotations

import json
import logging
from typing import Optional, Sequence

from training.common import TrainingConfig
from training.semi_supervised import run_pipeline

from ._cli import base_parser, to_config

LOGGER = logging.getLogger(__name__)


def parse_args(args: Optional[Sequence[str]] = None) -> TrainingConfig:
    return to_config(base_parser(__doc__, weak_required=True).parse_args(args=args), semi=True)


def main(args: Optional[Sequence[str]] = None) -> None:
    logging.basicConfig(level=logging.INFO, format="[%(asctime)s] %(levelname)s:%(name)s:%(message)s")
    config = parse_args(args)
    metrics = run_pipeline(config)
    LOGGER.info("Experiment complete. Metrics:\n%s", json.dumps(metrics, indent=2))


if __name__ == "__main__":  # pragma: no cover
    main()
