"""Shared training core — drop-in mirror of the reference's
src/training/common.py (same names, arguments, return values, artifacts and
error behaviour), running on the ssip HIP kernels.

What moved where (reference file:line -> here):
  TrainingConfig            common.py:45-80     same dataclass (+ dtype)
  set_seed                  common.py:87-93     same
  build_transforms          common.py:96-119    device transform specs (PIL decode + RNG
                                                draws stay in the worker, pixels on GPU)
  TransformSubset / Unlabeled / PseudoLabeled   common.py:126-194   same semantics
  stratified_split          common.py:197-224   same (sklearn train_test_split x2)
  make_balanced_sampler     common.py:227-246   same (WeightedRandomSampler)
  prepare_dataloaders       common.py:249-292   same loaders; uint8 batches + params
  create_model              common.py:299-304   SSIPResNet (torchvision init order/keys)
  train_model               common.py:345-432   same loop incl. the best_state alias quirk;
                                                device-side metric accumulation (one sync/epoch)
  evaluate_on_loader / evaluate_model / compute_accuracy_f1   common.py:307-342,439-506
  plots / confusion metrics / threshold selection             common.py:509-746
"""
from __future__ import annotations

import logging
import math
import os
import random
import sys
import warnings
from dataclasses import dataclass
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
from sklearn.metrics import (
    accuracy_score,
    auc,
    average_precision_score,
    confusion_matrix,
    precision_recall_curve,
    precision_recall_fscore_support,
    roc_curve,
)
from sklearn.model_selection import train_test_split
from torch.utils.data import DataLoader, Dataset, WeightedRandomSampler

_PKG = Path(__file__).resolve().parents[2]
if str(_PKG) not in sys.path:
    sys.path.insert(0, str(_PKG))

from ssip import SSIPResNet, ops, replace_fc  # noqa: E402
from ssip.data import Collate, DeviceTransformSpec, ImageFolder, pil_loader  # noqa: E402
from ssip.optim import AdamW  # noqa: E402
from ssip.resnet import DeviceImages  # noqa: E402

from . import distributed as D  # noqa: E402

LOGGER = logging.getLogger(__name__)

# ---------------------------------------------------------------------------
# Configuration (reference common.py:45-80)
# ---------------------------------------------------------------------------


@dataclass
class TrainingConfig:
    strong_data_dir: Path
    weak_data_dir: Path
    batch_size: int = 16
    val_split: float = 0.2
    test_split: float = 0.2
    seed: int = 42
    image_size: int = 224
    num_workers: int = 2
    device: str = "auto"
    positive_class: str = "cancer"
    target_recall: Optional[float] = None
    min_precision: Optional[float] = None
    max_fpr: Optional[float] = None
    f_beta: float = 2.0
    baseline_epochs: int = 10
    weak_pretrain_epochs: int = 5
    finetune_epochs: int = 8
    pseudo_label_threshold: float = 0.7
    learning_rate: float = 1e-4
    weight_decay: float = 1e-4
    early_stopping_patience: int = 3
    output_dir: Path = Path("outputs")
    results_table: Path = Path("outputs/tables/results_comparison.csv")
    baseline_curve_path: Path = Path("outputs/figures/train_curves_baseline.png")
    semi_curve_path: Path = Path("outputs/figures/train_curves_semi.png")
    baseline_confusion_path: Path = Path("outputs/figures/confusion_matrix_baseline.png")
    semi_confusion_path: Path = Path("outputs/figures/confusion_matrix_semi.png")
    roc_curve_path: Path = Path("outputs/figures/roc_curves.png")
    history_path: Path = Path("outputs/notes/training_history.json")
    baseline_checkpoint: Path = Path("outputs/models/baseline_resnet18.pt")
    semi_checkpoint: Path = Path("outputs/models/semi_resnet18.pt")
    unlabeled_cohort_csv: Optional[Path] = None
    operating_point_path: Path = Path("outputs/notes/operating_point.json")
    triage_csv_path: Path = Path("outputs/tables/unlabeled_predictions_semi.csv")
    # ssip extensions (optional, defaults keep reference numerics)
    dtype: str = "fp32"
    weights: Optional[Path] = None
    random_init: bool = False   # opt in to the seeded random backbone when no ImageNet weights are local
    consistency: bool = False   # semi stage = joint weak/strong consistency training (ssip.semi_step.SemiStep)
    lambda_u: float = 1.0       # weight of the unlabelled consistency term (--consistency)


# ---------------------------------------------------------------------------
# Reproducibility and transforms (reference common.py:87-119)
# ---------------------------------------------------------------------------


def set_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False


def build_transforms(image_size: int = 224) -> Dict[str, DeviceTransformSpec]:
    """train: Resize((S,S)) -> RandomHorizontalFlip -> RandomRotation(10) -> ToTensor -> Normalize;
    eval: Resize((S,S)) -> ToTensor -> Normalize — executed Pillow-exactly on the device."""
    return {"train": DeviceTransformSpec("train", image_size, degrees=10.0),
            "eval": DeviceTransformSpec("eval", image_size)}


def resolve_device(device: str) -> torch.device:
    """auto | cpu | cuda (reference semi_supervised.py:81-86); ssip runs on the HIP device only."""
    if device == "auto":
        if not torch.cuda.is_available():
            raise RuntimeError("ssip: no HIP device visible; this framework runs its compute on MI355X only")
        return D.setup(torch.device("cuda"))
    if device == "cpu":
        raise RuntimeError("ssip: --device cpu is not supported (the compute path is the HIP kernels); "
                           "use --device cuda or auto")
    return D.setup(torch.device(device))


# ---------------------------------------------------------------------------
# Datasets and loaders (reference common.py:126-292)
# ---------------------------------------------------------------------------


class TransformSubset(Dataset):
    def __init__(self, dataset: ImageFolder, indices: Sequence[int], transform=None, return_paths: bool = False):
        self.dataset = dataset
        self.indices = list(indices)
        self.transform = transform
        self.return_paths = return_paths

    def __len__(self) -> int:
        return len(self.indices)

    def __getitem__(self, idx: int):
        image, label = self.dataset[self.indices[idx]]
        if self.transform is not None:
            image = self.transform(image)
        if self.return_paths:
            return image, label, self.dataset.samples[self.indices[idx]][0]
        return image, label


class UnlabeledImageDataset(Dataset):
    def __init__(self, root_dir: Path, transform=None) -> None:
        self.root_dir = Path(root_dir)
        if not self.root_dir.exists():
            raise FileNotFoundError(f"Unlabeled directory not found: {self.root_dir}")
        self.image_paths = sorted(p for p in self.root_dir.iterdir()
                                  if p.suffix.lower() in {".jpg", ".jpeg", ".png", ".bmp"})
        self.transform = transform

    def __len__(self) -> int:
        return len(self.image_paths)

    def __getitem__(self, idx: int):
        path = self.image_paths[idx]
        image = pil_loader(path)
        if self.transform is not None:
            image = self.transform(image)
        return image, str(path)


class PseudoLabeledDataset(Dataset):
    def __init__(self, samples: Sequence[Tuple[str, int]], transform=None) -> None:
        self.samples = list(samples)
        self.transform = transform

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, idx: int):
        path, label = self.samples[idx]
        image = pil_loader(path)
        if self.transform is not None:
            image = self.transform(image)
        return image, label


def stratified_split(targets: Sequence[int], val_size: float, test_size: float, seed: int):
    """Two stratified train_test_split calls (reference common.py:197-224)."""
    indices = np.arange(len(targets))
    train_idx, temp_idx, _, temp_t = train_test_split(indices, targets, test_size=val_size + test_size,
                                                      random_state=seed, stratify=targets)
    val_idx, test_idx = train_test_split(temp_idx, test_size=test_size / (val_size + test_size),
                                         random_state=seed, stratify=temp_t)
    return np.array(train_idx), np.array(val_idx), np.array(test_idx)


def make_balanced_sampler(labels: Sequence[int]) -> WeightedRandomSampler:
    """Inverse-class-frequency weights with replacement (reference common.py:227-246)."""
    arr = np.array(labels)
    counts = np.bincount(arr)
    if len(np.nonzero(counts)[0]) < 2:
        LOGGER.warning("Only one class present in labels; using uniform sampling instead of balancing.")
        return WeightedRandomSampler(weights=[1.0] * int(len(arr)), num_samples=int(len(arr)), replacement=True)
    per_class = 1.0 / counts
    weights = per_class[arr].astype(float)
    return WeightedRandomSampler(weights=weights.tolist(), num_samples=int(len(weights)), replacement=True)


def _loader(ds, spec, batch_size, num_workers, sampler=None):
    return DataLoader(ds, batch_size=batch_size, sampler=sampler, shuffle=False, num_workers=num_workers,
                      pin_memory=torch.cuda.is_available(), collate_fn=Collate(spec))


def prepare_dataloaders(strong_data_dir: Path, transforms_map, batch_size: int, val_split: float, test_split: float,
                        seed: int, num_workers: int = 2):
    base = ImageFolder(strong_data_dir, transform=None)
    targets = np.array(base.targets)
    tr, va, te = stratified_split(targets.tolist(), val_split, test_split, seed)
    splits = {"train": tr, "val": va, "test": te}
    train_ds = TransformSubset(base, list(tr), transform=transforms_map["train"])
    val_ds = TransformSubset(base, list(va), transform=transforms_map["eval"], return_paths=True)
    test_ds = TransformSubset(base, list(te), transform=transforms_map["eval"], return_paths=True)
    sampler = make_balanced_sampler(targets[tr].tolist())
    if D.world() > 1:  # the same global draw on every rank, rank-strided
        sampler = D.RankStridedSampler(sampler)
    return (_loader(train_ds, transforms_map["train"], batch_size, num_workers, sampler),
            _loader(val_ds, transforms_map["eval"], batch_size, num_workers),
            _loader(test_ds, transforms_map["eval"], batch_size, num_workers),
            base, splits)


# ---------------------------------------------------------------------------
# Model and training loop (reference common.py:299-432)
# ---------------------------------------------------------------------------

_WEIGHTS_ENV = "SSIP_RESNET18_WEIGHTS"
_RANDOM_INIT_ENV = "SSIP_ALLOW_RANDOM_INIT"


def random_init_allowed(flag: bool = False) -> bool:
    return bool(flag) or os.environ.get(_RANDOM_INIT_ENV) == "1"


def create_model(num_classes: int, pretrained: bool = True, dtype: str = "fp32",
                 weights: Optional[Path] = None, allow_random_init: bool = False) -> SSIPResNet:
    """torchvision resnet18 (+ new fc) semantics and RNG consumption.  The
    ImageNet weights are a network download in the reference
    (ResNet18_Weights.IMAGENET1K_V1, common.py:299-304), which fails offline;
    here they load from `weights` or $SSIP_RESNET18_WEIGHTS (a torchvision
    state_dict).  Without either, pretrained=True raises like the
    reference's failed download, unless the caller opted in to the seeded
    random initialisation (allow_random_init / --random-init /
    $SSIP_ALLOW_RANDOM_INIT=1); the model then records it in `init_source`."""
    model = SSIPResNet("resnet18", num_classes=1000, dtype=dtype)
    model.init_source = "random_init"
    if pretrained:
        path = weights or os.environ.get(_WEIGHTS_ENV)
        if path and Path(path).exists():
            model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
            model.init_source = f"state_dict:{path}"
        elif random_init_allowed(allow_random_init):
            warnings.warn("ResNet18_Weights.IMAGENET1K_V1 unavailable offline; using the seeded random init "
                          "(opted in)")
            LOGGER.warning("Backbone: seeded random initialisation (no ImageNet weights; opted in)")
        else:
            raise RuntimeError(
                "ResNet18_Weights.IMAGENET1K_V1 is a network download and no local copy was given: pass --weights "
                f"<torchvision resnet18 state_dict> or set {_WEIGHTS_ENV}, or opt in to the seeded random "
                f"initialisation with --random-init (or {_RANDOM_INIT_ENV}=1)")
    replace_fc(model, num_classes)
    return model


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss (mean) with forward+backward fused in one HIP launch."""

    def forward(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        return _CE.apply(logits, labels)


class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss, dl, _ = ops.cross_entropy(logits.detach(), labels, want_grad=logits.requires_grad)
        ctx.save_for_backward(dl if dl is not None else torch.empty(0))
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def _to_device(inputs, device, model):
    if hasattr(inputs, "spec"):  # HostImageBatch
        return inputs.to(device, dtype=getattr(model, "compute_dtype", torch.float32))
    return inputs.to(device)


def compute_accuracy_f1(y_true: Sequence[int], y_pred: Sequence[int]) -> Tuple[float, float]:
    if len(y_true) == 0:
        return 0.0, 0.0
    acc = accuracy_score(y_true, y_pred)
    _, _, f1, _ = precision_recall_fscore_support(y_true, y_pred, average="binary", zero_division=0)
    return float(acc), float(f1)


def evaluate_on_loader(model: nn.Module, data_loader: DataLoader, criterion: nn.Module,
                       device: torch.device) -> Tuple[float, float, float]:
    model.eval()
    D.sync_buffers(model)  # under DP: every shard evaluated with rank 0's running statistics
    losses: List[torch.Tensor] = []
    y_true: List[torch.Tensor] = []
    y_pred: List[torch.Tensor] = []
    with torch.no_grad():
        for batch in D.shard_loader(data_loader):
            inputs, labels = batch[:2]
            inputs = _to_device(inputs, device, model)
            labels = labels.to(device)
            outputs = model(inputs)
            loss, _, pred = ops.cross_entropy(outputs, labels, want_grad=False)
            losses.append(loss)
            y_true.append(labels)
            y_pred.append(pred)
    # per-batch losses / predictions in batch order (gathered in rank order under DP)
    bl = D.gather_list(torch.cat(losses).cpu().numpy().astype(np.float64).tolist() if losses else [])
    yt = D.gather_list(torch.cat(y_true).cpu().numpy().tolist() if y_true else [])
    yp = D.gather_list(torch.cat(y_pred).cpu().numpy().tolist() if y_pred else [])
    avg = float(np.mean(bl)) if bl else 0.0
    acc, f1 = compute_accuracy_f1(yt, yp)
    return avg, acc, f1


def train_model(model: nn.Module, train_loader: DataLoader, val_loader: DataLoader, criterion: nn.Module,
                optimizer, device: torch.device, scheduler=None, num_epochs: int = 10,
                early_stopping_patience: int = 3, model_path: Optional[Path] = None):
    """Reference common.py:345-432, step for step (including
    `best_state = model.state_dict()` aliasing the live parameters, so the
    returned model is the LAST epoch while the checkpoint holds the best
    val-loss epoch).  Per-step losses/predictions stay on the device and are
    read once per epoch instead of three host syncs per step."""
    history: Dict[str, List[float]] = {k: [] for k in
                                       ("train_loss", "val_loss", "train_acc", "val_acc", "train_f1", "val_f1")}
    best_state = model.state_dict()
    best_val_loss = math.inf
    patience = 0
    for epoch in range(num_epochs):
        model.train()
        losses, yt, yp = [], [], []
        for inputs, labels in train_loader:
            inputs = _to_device(inputs, device, model)
            labels = labels.to(device)
            optimizer.zero_grad()
            outputs = model(inputs)
            loss = criterion(outputs, labels)
            loss.backward()
            optimizer.step()
            losses.append(loss.detach().view(1))
            yt.append(labels)
            yp.append(outputs.detach().argmax(dim=1))
        # under DP: rank 0's BN running statistics on every rank (DDP's buffer
        # broadcast) before the sharded validation pass and the checkpoint
        D.sync_buffers(model)
        # under DP the epoch's metrics cover every rank's steps (gathered in rank order)
        sl = D.gather_list(torch.cat(losses).cpu().numpy().astype(np.float64).tolist() if losses else [])
        tl = float(np.mean(sl)) if sl else 0.0
        ta, tf1 = compute_accuracy_f1(D.gather_list(torch.cat(yt).cpu().numpy().tolist() if yt else []),
                                      D.gather_list(torch.cat(yp).cpu().numpy().tolist() if yp else []))
        vl, va, vf1 = evaluate_on_loader(model, val_loader, criterion, device)
        if scheduler is not None:
            if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                scheduler.step(vl)
            else:
                scheduler.step()
        for k, v in zip(("train_loss", "val_loss", "train_acc", "val_acc", "train_f1", "val_f1"),
                        (tl, vl, ta, va, tf1, vf1)):
            history[k].append(v)
        LOGGER.info("Epoch %d/%d - train loss %.4f acc %.3f f1 %.3f | val loss %.4f acc %.3f f1 %.3f",
                    epoch + 1, num_epochs, tl, ta, tf1, vl, va, vf1)
        if vl < best_val_loss:
            best_val_loss = vl
            best_state = model.state_dict()
            patience = 0
            if model_path is not None and D.is_main():
                model_path.parent.mkdir(parents=True, exist_ok=True)
                torch.save(best_state, model_path)
        else:
            patience += 1
            if patience >= early_stopping_patience:
                LOGGER.info("Early stopping triggered at epoch %d", epoch + 1)
                break
    model.load_state_dict(best_state)
    return model, history


def make_optimizer(model: SSIPResNet, lr: float, weight_decay: float, params=None) -> AdamW:
    """optim.AdamW((p for p in model.parameters() if p.requires_grad), lr, wd) on the fused kernel."""
    arena = model.flatten_parameters()
    ps = [p for p in (params if params is not None else model.parameters()) if p.requires_grad]
    opt = AdamW(ps, lr=lr, weight_decay=weight_decay, arena=arena)
    D.attach_grad_allreduce(model, opt)  # no-op on one process
    return opt


# ---------------------------------------------------------------------------
# Evaluation helpers and plots (reference common.py:439-644)
# ---------------------------------------------------------------------------


def evaluate_model(model: nn.Module, data_loader: DataLoader, device: torch.device, pos_index: Optional[int] = None,
                   threshold: Optional[float] = None):
    model.eval()
    D.sync_buffers(model)
    y_true: List[int] = []
    y_pred: List[int] = []
    y_prob: List[float] = []
    paths_all: List[str] = []
    with torch.no_grad():
        for batch in D.shard_loader(data_loader):
            inputs, labels = batch[:2]
            extras = batch[2:] if len(batch) > 2 else []
            paths = extras[0] if extras else ["" for _ in range(len(labels))]
            inputs = _to_device(inputs, device, model)
            outputs = model(inputs)
            J = outputs.shape[1]
            pos_col = (1 if J > 1 else 0) if pos_index is None else pos_index
            _, _, amax, _, pos = ops.softmax_select(outputs, 0.0, pos_col)
            probs = pos.cpu().numpy()  # float32
            if threshold is None or J != 2:
                pred = amax.cpu().numpy()
            else:
                neg_col = 1 - pos_col
                pred = np.where(probs >= np.float32(threshold), pos_col, neg_col).astype(np.int64)
            y_true.extend(labels.numpy().tolist())
            y_pred.extend(pred.tolist())
            y_prob.extend(probs.tolist())
            paths_all.extend(str(p) for p in list(paths))
    if D.world() > 1:  # rank-ordered shards = the single-process order
        y_true, y_pred, y_prob, paths_all = (D.gather_list(v) for v in (y_true, y_pred, y_prob, paths_all))
    if pos_index is not None:
        ytb = (np.array(y_true) == pos_index).astype(int)
        ypb = (np.array(y_pred) == pos_index).astype(int)
        acc = accuracy_score(ytb, ypb)
        p, r, f1, _ = precision_recall_fscore_support(ytb, ypb, average="binary", zero_division=0)
    else:
        acc = accuracy_score(y_true, y_pred)
        p, r, f1, _ = precision_recall_fscore_support(y_true, y_pred, average="binary", zero_division=0)
    metrics = {"accuracy": float(acc), "precision": float(p), "recall": float(r), "f1": float(f1)}
    return metrics, np.array(y_true), np.array(y_pred), np.array(y_prob), paths_all


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def plot_training_curves(history: Dict[str, List[float]], output_path: Path, title: str) -> None:
    if not D.is_main():
        return
    plt = _plt()
    ep = range(1, len(history["train_loss"]) + 1)
    fig, ax = plt.subplots(1, 2, figsize=(10, 4))
    for key, lab in (("train_loss", "Train"), ("val_loss", "Validation")):
        ax[0].plot(ep, history[key], label=lab)
    ax[0].set(title=f"Loss - {title}", xlabel="Epoch", ylabel="Loss")
    ax[0].legend()
    for key, lab in (("train_f1", "Train"), ("val_f1", "Validation")):
        ax[1].plot(ep, history[key], label=lab)
    ax[1].set(title=f"F1 Score - {title}", xlabel="Epoch", ylabel="F1 Score")
    ax[1].legend()
    fig.tight_layout()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    fig.savefig(output_path, dpi=200)
    plt.close(fig)


def plot_confusion_matrix(y_true, y_pred, class_names: Sequence[str], output_path: Path) -> None:
    if not D.is_main():
        return
    plt = _plt()
    mat = confusion_matrix(y_true, y_pred)
    fig = plt.figure(figsize=(4, 4))
    plt.imshow(mat, interpolation="nearest", cmap="Blues")
    plt.title("Confusion Matrix")
    plt.colorbar()
    ticks = np.arange(len(class_names))
    plt.xticks(ticks, class_names, rotation=45)
    plt.yticks(ticks, class_names)
    half = mat.max() / 2.0 if mat.size else 0.5
    for i, j in np.ndindex(mat.shape):
        plt.text(j, i, format(mat[i, j], "d"), horizontalalignment="center",
                 color="white" if mat[i, j] > half else "black")
    plt.ylabel("True label")
    plt.xlabel("Predicted label")
    plt.tight_layout()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    fig.savefig(output_path, dpi=200)
    plt.close(fig)


def plot_roc_curves(curves: Dict[str, Tuple[np.ndarray, np.ndarray]], output_path: Path) -> None:
    if not D.is_main():
        return
    plt = _plt()
    fig = plt.figure(figsize=(6, 6))
    for label, (yt, yp) in curves.items():
        fpr, tpr, _ = roc_curve(yt, yp)
        plt.plot(fpr, tpr, label=f"{label} (AUC={auc(fpr, tpr):.3f})")
    plt.plot([0, 1], [0, 1], "k--", label="Chance")
    plt.xlabel("False Positive Rate")
    plt.ylabel("True Positive Rate")
    plt.title("ROC Curves")
    plt.legend(loc="lower right")
    plt.tight_layout()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    fig.savefig(output_path, dpi=200)
    plt.close(fig)


def plot_pr_curves(curves: Dict[str, Tuple[np.ndarray, np.ndarray]], output_path: Path) -> None:
    if not D.is_main():
        return
    plt = _plt()
    fig = plt.figure(figsize=(6, 6))
    for label, (yt, yp) in curves.items():
        prec, rec, _ = precision_recall_curve(yt, yp)
        plt.plot(rec, prec, label=f"{label} (AP={average_precision_score(yt, yp):.3f})")
    plt.xlabel("Recall")
    plt.ylabel("Precision")
    plt.title("Precision-Recall Curves")
    plt.legend(loc="lower left")
    plt.tight_layout()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    fig.savefig(output_path, dpi=200)
    plt.close(fig)


def compute_binary_confusion_metrics(y_true: np.ndarray, y_pred: np.ndarray, pos_index: int) -> Dict[str, float]:
    """Reference common.py:595-624."""
    yt = (np.asarray(y_true) == pos_index).astype(int)
    yp = (np.asarray(y_pred) == pos_index).astype(int)
    tp = float(((yt == 1) & (yp == 1)).sum())
    tn = float(((yt == 0) & (yp == 0)).sum())
    fp = float(((yt == 0) & (yp == 1)).sum())
    fn = float(((yt == 1) & (yp == 0)).sum())

    def ratio(a, b):
        return a / b if b > 0 else 0.0

    return {"TP": tp, "FP": fp, "TN": tn, "FN": fn, "TPR": ratio(tp, tp + fn), "TNR": ratio(tn, tn + fp),
            "FPR": ratio(fp, fp + tn), "FNR": ratio(fn, fn + tp), "precision": ratio(tp, tp + fp),
            "recall": ratio(tp, tp + fn), "accuracy": (tp + tn) / max(1, tp + tn + fp + fn)}


def plot_metrics_bars(metrics_map: Dict[str, Dict[str, float]], output_path: Path, keys: Sequence[str]) -> None:
    if not D.is_main():
        return
    plt = _plt()
    labels = list(metrics_map)
    x = np.arange(len(labels))
    w = 0.12
    fig = plt.figure(figsize=(max(7, len(labels) * 1.6), 4))
    for i, k in enumerate(keys):
        plt.bar(x + i * w, [metrics_map[lb].get(k, 0.0) for lb in labels], width=w, label=k)
    plt.xticks(x + (len(keys) - 1) * w / 2, labels, rotation=15)
    plt.ylabel("Score")
    plt.title("Metric Comparison")
    plt.ylim(0, 1.05)
    plt.legend()
    plt.tight_layout()
    output_path.parent.mkdir(parents=True, exist_ok=True)
    fig.savefig(output_path, dpi=200)
    plt.close(fig)


# ---------------------------------------------------------------------------
# Threshold selection (reference common.py:651-746)
# ---------------------------------------------------------------------------


def _binary_counts(y: np.ndarray, p: np.ndarray, thr: float):
    pred = (p >= thr).astype(int)
    tp = float(((y == 1) & (pred == 1)).sum())
    tn = float(((y == 0) & (pred == 0)).sum())
    fp = float(((y == 0) & (pred == 1)).sum())
    fn = float(((y == 1) & (pred == 0)).sum())
    return tp, tn, fp, fn


def find_threshold_for_target_recall(y_true_bin: np.ndarray, y_prob: np.ndarray, target_recall: float) -> float:
    """Largest candidate threshold whose recall reaches the target (scan from the top)."""
    y = np.asarray(y_true_bin)
    p = np.asarray(y_prob)
    if y.sum() == 0:
        return 0.5
    cands = np.unique(np.concatenate(([0.0], p)))
    best = cands[0]
    for thr in cands[::-1]:
        tp, _, _, fn = _binary_counts(y, p, thr)
        rec = tp / (tp + fn) if (tp + fn) > 0 else 0.0
        if rec >= target_recall:
            best = float(thr)
            break
    return float(best)


def select_operating_threshold(y_true_bin: np.ndarray, y_prob: np.ndarray, target_recall: float,
                               min_precision: Optional[float] = None, max_fpr: Optional[float] = None,
                               f_beta: float = 2.0) -> Tuple[float, Dict[str, Any]]:
    """Recall-first policy: constrained (largest feasible threshold) ->
    F-beta maximum -> recall-only -> minimum threshold."""
    y = np.asarray(y_true_bin)
    p = np.asarray(y_prob)
    if y.sum() == 0:
        return 0.5, {"policy": "no_positives", "recall": 0.0, "precision": 0.0, "fpr": 0.0}
    cands = np.unique(np.concatenate(([0.0], p, [1.0])))

    def stats(thr):
        tp, tn, fp, fn = _binary_counts(y, p, thr)
        rec = tp / (tp + fn) if (tp + fn) > 0 else 0.0
        prec = tp / (tp + fp) if (tp + fp) > 0 else 0.0
        fpr = fp / (fp + tn) if (fp + tn) > 0 else 0.0
        b2 = f_beta * f_beta
        fb = (1 + b2) * (prec * rec) / (b2 * prec + rec) if (prec + rec) > 0 else 0.0
        return rec, prec, fpr, fb

    feasible = []
    for thr in cands:
        rec, prec, fpr, _ = stats(thr)
        if rec + 1e-12 < target_recall:
            continue
        if min_precision is not None and prec + 1e-12 < min_precision:
            continue
        if max_fpr is not None and fpr - 1e-12 > max_fpr:
            continue
        feasible.append((float(thr), rec, prec, fpr))
    if feasible:
        thr, rec, prec, fpr = max(feasible, key=lambda t: t[0])
        return float(thr), {"policy": "constrained", "recall": float(rec), "precision": float(prec),
                            "fpr": float(fpr)}
    scored = [(stats(t)[3], float(t)) for t in cands]
    fb, thr = max(scored, key=lambda t: (t[0], t[1]))
    if fb > 0:
        rec, prec, fpr, _ = stats(thr)
        return float(thr), {"policy": "fbeta", "fbeta": float(fb), "recall": float(rec), "precision": float(prec),
                            "fpr": float(fpr)}
    t = find_threshold_for_target_recall(y, p, target_recall)
    rec, prec, fpr, _ = stats(t)
    return float(t), {"policy": "recall_only", "recall": float(rec), "precision": float(prec), "fpr": float(fpr)}
