"""Supervised (baseline) pipeline — drop-in mirror of the reference's
src/training/supervised.py:38-144 on the ssip kernels."""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Dict

import pandas as pd
import torch

from . import distributed as D
from .common import (
    CrossEntropyLoss,
    TrainingConfig,
    build_transforms,
    create_model,
    evaluate_model,
    make_optimizer,
    plot_confusion_matrix,
    plot_pr_curves,
    plot_roc_curves,
    plot_training_curves,
    prepare_dataloaders,
    resolve_device,
    select_operating_threshold,
    set_seed,
    train_model,
)

LOGGER = logging.getLogger(__name__)


def run_supervised(config: TrainingConfig) -> Dict[str, Dict[str, float]]:
    set_seed(config.seed)
    device = resolve_device(config.device)
    LOGGER.info("Using device: %s", device)
    tfm = build_transforms(config.image_size)
    train_loader, val_loader, test_loader, base, _ = prepare_dataloaders(
        config.strong_data_dir, tfm, config.batch_size, config.val_split, config.test_split, config.seed,
        config.num_workers)
    if config.positive_class not in base.class_to_idx:
        raise ValueError(f"Positive class '{config.positive_class}' not found in dataset classes: {base.classes}")
    pos_index = int(base.class_to_idx[config.positive_class])
    model = create_model(len(base.classes), pretrained=True, dtype=config.dtype, weights=config.weights,
                           allow_random_init=config.random_init).to(device)
    criterion = CrossEntropyLoss()
    opt = make_optimizer(model, config.learning_rate, config.weight_decay)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", patience=2, factor=0.5)
    model, history = train_model(model, train_loader, val_loader, criterion, opt, device, scheduler=sch,
                                 num_epochs=config.baseline_epochs,
                                 early_stopping_patience=config.early_stopping_patience,
                                 model_path=config.baseline_checkpoint)
    arg_metrics, a_true, a_pred, a_prob, _ = evaluate_model(model, test_loader, device)
    if config.target_recall is not None:
        _, yv, _, pv, _ = evaluate_model(model, val_loader, device, pos_index=pos_index)
        thr, meta = select_operating_threshold((yv == pos_index).astype(int), pv,
                                               target_recall=float(config.target_recall),
                                               min_precision=config.min_precision, max_fpr=config.max_fpr,
                                               f_beta=config.f_beta)
        thr_metrics, t_true, t_pred, t_prob, _ = evaluate_model(model, test_loader, device, pos_index=pos_index,
                                                                threshold=thr)
        thr_metrics.update(threshold=float(thr), target_recall=float(config.target_recall),
                           min_precision=None if config.min_precision is None else float(config.min_precision),
                           max_fpr=None if config.max_fpr is None else float(config.max_fpr),
                           threshold_policy=meta.get("policy", "unknown"))
    else:
        thr_metrics = dict(arg_metrics)
        t_true, t_pred, t_prob = a_true, a_pred, a_prob
        thr_metrics.update(threshold=None, target_recall=None, min_precision=None, max_fpr=None,
                           threshold_policy="disabled")
    plot_training_curves(history, config.baseline_curve_path, "Baseline")
    plot_confusion_matrix(a_true, a_pred, base.classes, config.baseline_confusion_path)
    yb = (t_true == pos_index).astype(int)
    plot_roc_curves({"Baseline": (yb, t_prob)}, config.roc_curve_path)
    plot_pr_curves({"Baseline": (yb, t_prob)}, Path("outputs/figures/pr_curves_baseline.png"))
    if D.is_main():
        config.results_table.parent.mkdir(parents=True, exist_ok=True)
        pd.DataFrame.from_dict({"baseline_thresholded": thr_metrics}, orient="index").to_csv(config.results_table)
    return {"baseline_thresholded": thr_metrics, "baseline_argmax": arg_metrics}
