"""Semi-supervised pipeline — drop-in mirror of the reference's
src/training/semi_supervised.py: baseline -> pseudo-label the unlabelled pool
-> frozen-backbone pretrain on pseudo-labels -> unfreeze + fine-tune ->
evaluate / threshold -> artifacts, with the compute on the ssip kernels.

Reference map: generate_pseudo_labels :44-72, run_pipeline :75-516 (stages
:103-311, artifacts :360-511; the hard-coded `outputs/...` paths are kept).
"""
from __future__ import annotations

import json
import logging
import time
from pathlib import Path
from typing import Any, Dict, List, Tuple

import numpy as np
import pandas as pd
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from ssip import ops
from ssip.data import Collate

from . import distributed as D
from .common import (
    CrossEntropyLoss,
    PseudoLabeledDataset,
    TrainingConfig,
    UnlabeledImageDataset,
    _to_device,
    build_transforms,
    compute_binary_confusion_metrics,
    create_model,
    evaluate_model,
    make_balanced_sampler,
    make_optimizer,
    plot_confusion_matrix,
    plot_metrics_bars,
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


def generate_pseudo_labels(model: nn.Module, data_loader: DataLoader, device: torch.device,
                           threshold: float = 0.7) -> List[Tuple[str, int, float]]:
    """(path, argmax, confidence) for every image whose max softmax >= threshold
    (reference semi_supervised.py:44-72); softmax/max/threshold in one kernel,
    one device->host copy per batch."""
    model.eval()
    D.sync_buffers(model)  # under DP: every shard labelled by rank 0's model
    out: List[Tuple[str, int, float]] = []
    with torch.no_grad():
        for images, paths in D.shard_loader(data_loader):
            images = _to_device(images, device, model)
            logits = model(images)
            _, conf, pred, keep, _ = ops.softmax_select(logits, float(threshold), 0)
            c = conf.cpu().numpy()
            pr = pred.cpu().numpy()
            for path, p, cf in zip(paths, pr, c):
                if cf >= np.float32(threshold):
                    out.append((path, int(p), float(cf)))
    out = D.gather_list(out)  # rank-ordered shards of the pool = the single-process order
    LOGGER.info("Generated %d pseudo-labelled samples with threshold %.2f", len(out), threshold)
    return out


def _threshold_block(model, val_loader, test_loader, device, pos_index, cfg: TrainingConfig, arg_metrics,
                     arg_true, arg_pred, arg_prob, train_time):
    if cfg.target_recall is not None:
        _, yv, _, pv, _ = evaluate_model(model, val_loader, device, pos_index=pos_index)
        thr, meta = select_operating_threshold((yv == pos_index).astype(int), pv, target_recall=float(cfg.target_recall),
                                               min_precision=cfg.min_precision, max_fpr=cfg.max_fpr,
                                               f_beta=cfg.f_beta)
        m, yt, yp, pp, _ = evaluate_model(model, test_loader, device, pos_index=pos_index, threshold=thr)
        m["threshold"] = float(thr)
        m["target_recall"] = float(cfg.target_recall)
        m["min_precision"] = None if cfg.min_precision is None else float(cfg.min_precision)
        m["max_fpr"] = None if cfg.max_fpr is None else float(cfg.max_fpr)
        m["threshold_policy"] = meta.get("policy", "unknown")
    else:
        thr = None
        m = dict(arg_metrics)
        yt, yp, pp = arg_true, arg_pred, arg_prob
        m.update(threshold=None, target_recall=None, min_precision=None, max_fpr=None, threshold_policy="disabled")
    m["training_time_sec"] = train_time
    return thr, m, yt, yp, pp


def _filter_cohort(ds: UnlabeledImageDataset, cfg: TrainingConfig) -> None:
    """Restrict the pool to the cohort CSV's `path` column (reference :191-228)."""
    cohort = Path(cfg.unlabeled_cohort_csv)
    if not cohort.exists():
        raise FileNotFoundError(f"Cohort CSV not found: {cohort}")
    df = pd.read_csv(cohort)
    if "path" not in df.columns:
        raise ValueError("Cohort CSV must contain a 'path' column")
    allowed = set()
    weak = cfg.weak_data_dir.name
    for s in df["path"].astype(str).tolist():
        pp = Path(s)
        cands = set()
        if pp.is_absolute():
            cands.add(pp.resolve())
        else:
            cands.add((cfg.weak_data_dir / pp).resolve())
            if len(pp.parts) > 1 and pp.parts[0] == weak:
                cands.add((cfg.weak_data_dir / Path(*pp.parts[1:])).resolve())
            if len(pp.parts) == 1:
                cands.add((cfg.weak_data_dir / pp.name).resolve())
        allowed.update(str(c) for c in cands)
    before = len(ds.image_paths)
    ds.image_paths = [Path(p) for p in ds.image_paths if str(Path(p).resolve()) in allowed]
    after = len(ds.image_paths)
    LOGGER.info("Filtered unlabeled pool via cohort CSV: %d -> %d images (%d excluded)", before, after, before - after)
    if after == 0:
        raise RuntimeError("Cohort filtering removed all unlabeled images; check the CSV paths match --weak-data-dir.")


class _Raw:
    """uint8 pixels of a dataset's images (decode only; the consistency step
    draws and applies its own weak / strong views on the device)."""

    def __init__(self, paths_labels):
        self.items = list(paths_labels)

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        from ssip.data import pil_loader

        path, label = self.items[i]
        return torch.from_numpy(np.ascontiguousarray(np.asarray(pil_loader(path)))), label


def _stack(batch):
    imgs = [b[0] for b in batch]
    if len({tuple(t.shape) for t in imgs}) != 1:
        raise ValueError("--consistency needs equally sized images within a batch")
    return torch.stack(imgs), torch.tensor([b[1] for b in batch], dtype=torch.int64)


def train_consistency(model, base, train_idx, pool, val_loader, criterion, device, config: TrainingConfig):
    """Joint weak/strong consistency training (ssip.semi_step.SemiStep, the
    benchmarked step) for config.weak_pretrain_epochs epochs: each step pairs
    a balanced-sampled labelled batch with the next unlabelled batch of the
    pool; tau = --pseudo-threshold (reference rule, semi_supervised.py:60-66),
    loss = CE(labelled) + lambda_u * mean_u[mask * CE(strong, pseudo)].  The
    history has the reference's six keys (train_* over the labelled part)."""
    from ssip.dist import GradBucketer
    from ssip.semi_step import SemiStep

    from .common import compute_accuracy_f1, evaluate_on_loader

    D.broadcast_model(model)  # rank 0's initial weights and buffers on every rank
    bucketer = GradBucketer(model.flatten_parameters()) if D.world() > 1 else None
    step = SemiStep(model, lr=config.learning_rate, weight_decay=config.weight_decay,
                    tau=config.pseudo_label_threshold, lambda_u=config.lambda_u, image_size=config.image_size,
                    bucketer=bucketer, seed=config.seed + D.rank())
    bs = config.batch_size
    lab = _Raw([base.samples[int(i)] for i in train_idx])
    sampler = make_balanced_sampler([base.samples[int(i)][1] for i in train_idx])
    if D.world() > 1:
        sampler = D.RankStridedSampler(sampler)
    lab_loader = DataLoader(lab, batch_size=bs, sampler=sampler, num_workers=config.num_workers, collate_fn=_stack,
                            drop_last=True)
    unl = _Raw([(str(p), -1) for p in pool.image_paths])
    gen = torch.Generator().manual_seed(config.seed)
    history: Dict[str, List[float]] = {k: [] for k in
                                       ("train_loss", "val_loss", "train_acc", "val_acc", "train_f1", "val_f1")}
    for epoch in range(config.weak_pretrain_epochs):
        model.train()
        order = torch.randperm(len(unl), generator=gen).tolist()
        # every rank runs the same number of steps (each step all-reduces gradients)
        unl_loader = D.shard_loader(DataLoader(torch.utils.data.Subset(unl, order), batch_size=bs, shuffle=False,
                                               num_workers=config.num_workers, collate_fn=_stack, drop_last=True),
                                    even=True)
        lab_iter = iter(lab_loader)
        losses, yt, yp = [], [], []
        padded = getattr(unl_loader, "ssip_padded", None)
        for bi, (xu, _) in enumerate(unl_loader):
            try:
                xl, yl = next(lab_iter)
            except StopIteration:
                lab_iter = iter(lab_loader)
                xl, yl = next(lab_iter)
            out = step(xl.to(device, non_blocking=True), yl.to(device), xu.to(device, non_blocking=True))
            if padded is not None and padded[bi]:
                continue  # a wrap-around repeat (shard_loader even=True): stepped, not averaged
            losses.append(out.loss[0:1].clone())
            yt.append(yl)
            yp.append(step.last["logits"][: yl.shape[0]].argmax(1).cpu())
        D.sync_buffers(model)  # rank 0's running statistics before the sharded validation pass
        sl = D.gather_list(torch.cat(losses).cpu().double().tolist() if losses else [])
        tl = float(np.mean(sl)) if sl else 0.0
        ta, tf1 = compute_accuracy_f1(D.gather_list(torch.cat(yt).tolist() if yt else []),
                                      D.gather_list(torch.cat(yp).tolist() if yp else []))
        vl, va, vf1 = evaluate_on_loader(model, val_loader, criterion, device)
        for k, v in zip(("train_loss", "val_loss", "train_acc", "val_acc", "train_f1", "val_f1"),
                        (tl, vl, ta, va, tf1, vf1)):
            history[k].append(v)
        LOGGER.info("Consistency epoch %d/%d - train loss %.4f acc %.3f | val loss %.4f acc %.3f f1 %.3f",
                    epoch + 1, config.weak_pretrain_epochs, tl, ta, vl, va, vf1)
    model.grad_ready_hook = None
    return history


def run_pipeline(config: TrainingConfig) -> Dict[str, Dict[str, float]]:
    set_seed(config.seed)
    device = resolve_device(config.device)
    LOGGER.info("Using device: %s", device)
    tfm = build_transforms(config.image_size)
    train_loader, val_loader, test_loader, base, splits = prepare_dataloaders(
        config.strong_data_dir, tfm, config.batch_size, config.val_split, config.test_split, config.seed,
        config.num_workers)
    num_classes = len(base.classes)
    if config.positive_class not in base.class_to_idx:
        raise ValueError(f"Positive class '{config.positive_class}' not found in dataset classes: {base.classes}")
    pos_index = int(base.class_to_idx[config.positive_class])
    criterion = CrossEntropyLoss()

    # baseline
    baseline = create_model(num_classes, pretrained=True, dtype=config.dtype, weights=config.weights,
                           allow_random_init=config.random_init).to(device)
    opt = make_optimizer(baseline, config.learning_rate, config.weight_decay)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", patience=2, factor=0.5)
    t0 = time.time()
    baseline, base_hist = train_model(baseline, train_loader, val_loader, criterion, opt, device, scheduler=sch,
                                      num_epochs=config.baseline_epochs,
                                      early_stopping_patience=config.early_stopping_patience,
                                      model_path=config.baseline_checkpoint)
    base_time = time.time() - t0
    b_arg, b_true, b_pred, b_prob, _ = evaluate_model(baseline, test_loader, device)
    thr_b, b_thr, bt_true, bt_pred, bt_prob = _threshold_block(baseline, val_loader, test_loader, device, pos_index,
                                                               config, b_arg, b_true, b_pred, b_prob, base_time)
    plot_training_curves(base_hist, config.baseline_curve_path, "Baseline")

    # pseudo-labelling over the unlabelled pool
    pool = UnlabeledImageDataset(config.weak_data_dir, transform=tfm["eval"])
    if config.unlabeled_cohort_csv is not None:
        _filter_cohort(pool, config)
    pool_loader = DataLoader(pool, batch_size=config.batch_size, shuffle=False, num_workers=config.num_workers,
                             pin_memory=torch.cuda.is_available(), collate_fn=Collate(tfm["eval"]))
    pseudo = generate_pseudo_labels(baseline, pool_loader, device, config.pseudo_label_threshold)
    pseudo_ds = PseudoLabeledDataset([(p, l) for p, l, _ in pseudo], transform=tfm["train"])
    if len(pseudo_ds) == 0:
        raise RuntimeError("No pseudo-labelled samples were generated. Try lowering the threshold.")
    pseudo_sampler = make_balanced_sampler([l for _, l, _ in pseudo])
    if D.world() > 1:
        pseudo_sampler = D.RankStridedSampler(pseudo_sampler)
    pseudo_loader = DataLoader(pseudo_ds, batch_size=config.batch_size, sampler=pseudo_sampler,
                               num_workers=config.num_workers, pin_memory=torch.cuda.is_available(),
                               collate_fn=Collate(tfm["train"]))

    # frozen-backbone pretrain (BN still in train mode), then fine-tune
    semi = create_model(num_classes, pretrained=True, dtype=config.dtype, weights=config.weights,
                           allow_random_init=config.random_init).to(device)
    t0 = time.time()
    if config.consistency:
        # build extension (BASELINE config 3): joint consistency training in place of the pretrain
        pre_hist = train_consistency(semi, base, splits["train"], pool, val_loader, criterion, device, config)
    else:
        for name, p in semi.named_parameters():
            if not name.startswith("fc"):
                p.requires_grad = False
        opt_p = make_optimizer(semi, config.learning_rate, config.weight_decay)
        sch_p = torch.optim.lr_scheduler.ReduceLROnPlateau(opt_p, mode="min", patience=2, factor=0.5)
        semi, pre_hist = train_model(semi, pseudo_loader, val_loader, criterion, opt_p, device, scheduler=sch_p,
                                     num_epochs=config.weak_pretrain_epochs,
                                     early_stopping_patience=config.early_stopping_patience)
    for p in semi.parameters():
        p.requires_grad = True
    opt_f = make_optimizer(semi, config.learning_rate / 2, config.weight_decay)
    sch_f = torch.optim.lr_scheduler.ReduceLROnPlateau(opt_f, mode="min", patience=2, factor=0.5)
    semi, fin_hist = train_model(semi, train_loader, val_loader, criterion, opt_f, device, scheduler=sch_f,
                                 num_epochs=config.finetune_epochs,
                                 early_stopping_patience=config.early_stopping_patience,
                                 model_path=config.semi_checkpoint)
    semi_time = time.time() - t0
    s_arg, s_true, s_pred, s_prob, _ = evaluate_model(semi, test_loader, device)
    thr_s, s_thr, st_true, st_pred, st_prob = _threshold_block(semi, val_loader, test_loader, device, pos_index,
                                                               config, s_arg, s_true, s_pred, s_prob, semi_time)

    # artifacts (reference :360-511)
    payload = {"baseline": base_hist, "semi_pretrain": pre_hist, "semi_finetune": fin_hist,
               "splits": {k: v.tolist() for k, v in splits.items()}, "pseudo_label_count": len(pseudo)}
    if D.is_main():
        config.history_path.parent.mkdir(parents=True, exist_ok=True)
        with open(config.history_path, "w", encoding="utf-8") as fp:
            json.dump(payload, fp, indent=2)
    joined = {k: pre_hist[k] + fin_hist[k] for k in pre_hist}
    plot_training_curves(joined, config.semi_curve_path, "Semi-supervised")
    plot_confusion_matrix(b_true, b_pred, base.classes, config.baseline_confusion_path)
    plot_confusion_matrix(bt_true, bt_pred, base.classes, Path("outputs/figures/confusion_matrix_baseline_thresholded.png"))
    plot_confusion_matrix(s_true, s_pred, base.classes, config.semi_confusion_path)
    plot_confusion_matrix(st_true, st_pred, base.classes, Path("outputs/figures/confusion_matrix_semi_thresholded.png"))
    yb = (bt_true == pos_index).astype(int)
    ys = (st_true == pos_index).astype(int)
    plot_roc_curves({"Baseline": (yb, bt_prob), "Semi-supervised": (ys, st_prob)}, config.roc_curve_path)
    plot_pr_curves({"Baseline": (yb, bt_prob), "Semi-supervised": (ys, st_prob)}, Path("outputs/figures/pr_curves.png"))

    rows: Dict[str, Dict[str, Any]] = {}
    rows["baseline_argmax"] = compute_binary_confusion_metrics(b_true, b_pred, pos_index) | {
        "threshold": None, "target_recall": None, "training_time_sec": b_arg.get("training_time_sec", base_time)}
    rows["baseline_thresholded"] = compute_binary_confusion_metrics(bt_true, bt_pred, pos_index) | {
        "threshold": None if thr_b is None else float(thr_b),
        "target_recall": None if config.target_recall is None else float(config.target_recall),
        "training_time_sec": b_thr.get("training_time_sec", base_time),
        "min_precision": b_thr.get("min_precision"), "max_fpr": b_thr.get("max_fpr")}
    rows["semi_argmax"] = compute_binary_confusion_metrics(s_true, s_pred, pos_index) | {
        "threshold": None, "target_recall": None, "training_time_sec": s_arg.get("training_time_sec", semi_time)}
    rows["semi_thresholded"] = compute_binary_confusion_metrics(st_true, st_pred, pos_index) | {
        "threshold": None if thr_s is None else float(thr_s),
        "target_recall": None if config.target_recall is None else float(config.target_recall),
        "training_time_sec": s_thr.get("training_time_sec", semi_time),
        "min_precision": s_thr.get("min_precision"), "max_fpr": s_thr.get("max_fpr")}
    if D.is_main():
        Path("outputs/tables").mkdir(parents=True, exist_ok=True)
        pd.DataFrame.from_dict(rows, orient="index").to_csv(Path("outputs/tables/results_comparison_detailed.csv"))
        config.results_table.parent.mkdir(parents=True, exist_ok=True)
        pd.DataFrame.from_dict({"baseline_thresholded": b_thr, "semi_thresholded": s_thr},
                               orient="index").to_csv(config.results_table)
    plot_metrics_bars(rows, Path("outputs/figures/metrics_comparison.png"),
                      keys=["TPR", "FPR", "TNR", "precision", "accuracy"])

    try:
        op = {"model": "semi_supervised_resnet18", "checkpoint": str(config.semi_checkpoint),
              "positive_class": config.positive_class, "threshold": s_thr.get("threshold"),
              "policy": s_thr.get("threshold_policy"), "target_recall": config.target_recall,
              "min_precision": config.min_precision, "max_fpr": config.max_fpr, "seed": config.seed}
        if D.is_main():
            config.operating_point_path.parent.mkdir(parents=True, exist_ok=True)
            with open(config.operating_point_path, "w", encoding="utf-8") as fp:
                json.dump(op, fp, indent=2)
    except Exception as exc:  # reference: warn and continue
        LOGGER.warning("Failed to write operating_point.json: %s", exc)

    try:
        tthr = s_thr.get("threshold")
        if tthr is not None:
            tri_loader = DataLoader(pool, batch_size=config.batch_size, shuffle=False,
                                    num_workers=config.num_workers, pin_memory=torch.cuda.is_available(),
                                    collate_fn=Collate(tfm["eval"]))
            semi.eval()
            D.sync_buffers(semi)
            recs = []
            with torch.no_grad():
                for images, paths in D.shard_loader(tri_loader):
                    logits = semi(_to_device(images, device, semi))
                    _, _, _, _, pos = ops.softmax_select(logits, 0.0, pos_index)
                    for pth, pr in zip(paths, pos.cpu().numpy().tolist()):
                        recs.append({"path": str(pth), "prob_positive": float(pr), "flagged": bool(pr >= float(tthr))})
            df = pd.DataFrame(D.gather_list(recs))
            if D.is_main():
                config.triage_csv_path.parent.mkdir(parents=True, exist_ok=True)
                df.to_csv(config.triage_csv_path, index=False)
            LOGGER.info("Wrote triage CSV with %d rows (%d flagged) to %s", len(df),
                        int(df["flagged"].sum()) if not df.empty else 0, config.triage_csv_path)
        else:
            LOGGER.info("Skipping triage CSV: no threshold selected (thresholding disabled)")
    except Exception as exc:
        LOGGER.warning("Failed to write triage CSV: %s", exc)

    return {"baseline_thresholded": b_thr, "semi_thresholded": s_thr}
