"""Argument surface shared by the two training CLIs (reference
src/semi_supervised_training.py:521-637, src/supervised_training.py:23-111)."""
from __future__ import annotations

import argparse
from pathlib import Path

from training.common import TrainingConfig


def base_parser(doc: str, weak_required: bool) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=doc)
    p.add_argument("--strong-data-dir", type=Path, required=True,
                   help="Path to the strongly labelled dataset (ImageFolder layout).")
    if weak_required:
        p.add_argument("--weak-data-dir", type=Path, required=True,
                       help="Path to the weakly labelled/unlabelled dataset (flat directory).")
    else:
        p.add_argument("--weak-data-dir", type=Path, default=Path("unused"),
                       help="Unused placeholder for compatibility with TrainingConfig.")
    p.add_argument("--batch-size", type=int, default=16)
    p.add_argument("--val-split", type=float, default=0.2)
    p.add_argument("--test-split", type=float, default=0.2)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-workers", type=int, default=2, help="Dataloader worker processes")
    p.add_argument("--baseline-epochs", type=int, default=10)
    if weak_required:
        p.add_argument("--weak-pretrain-epochs", type=int, default=5)
        p.add_argument("--finetune-epochs", type=int, default=8)
        p.add_argument("--pseudo-threshold", type=float, default=0.7)
    p.add_argument("--learning-rate", type=float, default=1e-4)
    p.add_argument("--weight-decay", type=float, default=1e-4)
    p.add_argument("--early-stopping", type=int, default=3)
    p.add_argument("--positive-class", type=str, default="cancer",
                   help="Name of the positive class (matching labeled folder name)")
    p.add_argument("--target-recall", type=float, default=None,
                   help="Optional target recall for validation-based threshold selection (0-1).")
    p.add_argument("--min-precision", type=float, default=None)
    p.add_argument("--max-fpr", type=float, default=None)
    p.add_argument("--f-beta", type=float, default=2.0)
    p.add_argument("--device", type=str, default="auto", choices=["auto", "cpu", "cuda"],
                   help="Device to use: auto (default), cpu, or cuda")
    p.add_argument("--output-dir", type=Path, default=Path("outputs"), help="Base directory for experiment artefacts.")
    if weak_required:
        p.add_argument("--unlabeled-cohort-csv", type=Path, default=None,
                       help="Optional CSV listing unlabeled image paths to include in pseudo-labeling (column: path).")
        p.add_argument("--consistency", action="store_true",
                       help="Replace the frozen-backbone pseudo-label pretrain with joint consistency training "
                            "(labelled CE + lambda * masked CE of strong views on weak-view pseudo-labels, "
                            "--pseudo-threshold as tau) for --weak-pretrain-epochs epochs (BASELINE config 3).")
        p.add_argument("--lambda-u", type=float, default=1.0, help="Consistency-loss weight (--consistency).")
    # ssip extensions (optional)
    p.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16"],
                   help="Activation dtype of the HIP kernels (fp32 = reference numerics, bf16 = throughput).")
    p.add_argument("--weights", type=Path, default=None,
                   help="Local torchvision resnet18 state_dict standing in for the IMAGENET1K_V1 download.")
    p.add_argument("--random-init", action="store_true",
                   help="Allow the seeded random backbone when no ImageNet weights are available locally "
                        "(otherwise a missing download is an error, as in the reference).")
    return p


def to_config(a, semi: bool) -> TrainingConfig:
    o = a.output_dir
    return TrainingConfig(
        strong_data_dir=a.strong_data_dir, weak_data_dir=a.weak_data_dir, batch_size=a.batch_size,
        val_split=a.val_split, test_split=a.test_split, seed=a.seed, image_size=a.image_size,
        num_workers=a.num_workers, positive_class=a.positive_class, target_recall=a.target_recall,
        min_precision=a.min_precision, max_fpr=a.max_fpr, f_beta=a.f_beta, baseline_epochs=a.baseline_epochs,
        weak_pretrain_epochs=a.weak_pretrain_epochs if semi else 0,
        finetune_epochs=a.finetune_epochs if semi else 0,
        pseudo_label_threshold=a.pseudo_threshold if semi else 0.0,
        learning_rate=a.learning_rate, weight_decay=a.weight_decay, early_stopping_patience=a.early_stopping,
        device=a.device, output_dir=o,
        results_table=o / "tables/results_comparison.csv",
        baseline_curve_path=o / "figures/train_curves_baseline.png",
        semi_curve_path=o / "figures/train_curves_semi.png",
        baseline_confusion_path=o / "figures/confusion_matrix_baseline.png",
        semi_confusion_path=o / "figures/confusion_matrix_semi.png",
        roc_curve_path=o / "figures/roc_curves.png",
        history_path=o / "notes/training_history.json",
        baseline_checkpoint=o / "models/baseline_resnet18.pt",
        semi_checkpoint=o / "models/semi_resnet18.pt",
        unlabeled_cohort_csv=a.unlabeled_cohort_csv if semi else None,
        dtype=a.dtype, weights=a.weights, random_init=a.random_init,
        consistency=bool(getattr(a, "consistency", False)) if semi else False,
        lambda_u=float(getattr(a, "lambda_u", 1.0)),
    )
