"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's
own Python (Septimus4/semi-supervised-image-processing, read-only at
/root/reference) on CPU in the build container.

torchvision is not installed in this image, so `import torchvision` is
served by the oracle's restatement (oracle/torchvision_restate/), which
delegates every image op to Pillow exactly as torchvision does.  Nothing in
this script runs on the GPU box (it needs /root/reference); the fixtures it
writes are small data files (inputs and expected outputs).

Run:  python tests/golden/make_goldens.py            (everything)
      python tests/golden/make_goldens.py --only real  (section 11 only)
"""
from __future__ import annotations

import json
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
ROOT = OUT.parents[1]


def main() -> None:
    if not REF.exists():
        sys.exit("make_goldens: /root/reference not present (fixtures are generated in the build container only)")
    sys.path.insert(0, str(ROOT / "oracle" / "torchvision_restate"))
    sys.path.insert(0, str(REF / "src"))
    sys.path.insert(0, str(REF))
    import torch
    from PIL import Image
    from torch.utils.data import DataLoader, Dataset

    from training import common as C  # reference module
    from training import semi_supervised as SS  # reference module
    import src.feature_extraction as FE  # reference module

    # 11. the reference's run_supervised on its own labelled MRI set at 224^2
    #     (prediction-level parity on the real val/test split)
    _real_supervised(C)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "real":
        return

    data = REF / "mri_dataset_brain_cancer_oc"
    goldens = {}

    # 1. stratified split on the real labelled set (seed 42 = default; and 7)
    import torchvision

    base = torchvision.datasets.ImageFolder(data / "avec_labels")
    targets = list(base.targets)
    splits = {}
    for seed in (42, 7):
        tr, va, te = C.stratified_split(targets, 0.2, 0.2, seed)
        splits[str(seed)] = {"train": tr.tolist(), "val": va.tolist(), "test": te.tolist()}
    goldens["splits"] = {"targets": targets, "classes": base.classes,
                         "samples": [str(Path(p).relative_to(data)) for p, _ in base.samples], "by_seed": splits}
    # a synthetic, unbalanced case
    tgt2 = [0] * 30 + [1] * 70
    tr, va, te = C.stratified_split(tgt2, 0.15, 0.25, 3)
    goldens["splits"]["synthetic"] = {"targets": tgt2, "val": 0.15, "test": 0.25, "seed": 3,
                                      "train": tr.tolist(), "val_idx": va.tolist(), "test_idx": te.tolist()}

    # 2. balanced sampler: weights + draws under a fixed seed
    samp = []
    for labels, seed in (([0, 1, 1, 1, 0, 1, 1, 1, 1, 0], 5), ([1] * 12, 9), ([0] * 3 + [1] * 9, 11)):
        s = C.make_balanced_sampler(labels)
        torch.manual_seed(seed)
        draws = list(iter(s))
        samp.append({"labels": labels, "seed": seed, "weights": [float(w) for w in s.weights.tolist()],
                     "num_samples": s.num_samples, "draws": [int(d) for d in draws]})
    goldens["sampler"] = samp

    # 3. threshold selection / metrics on seeded probability vectors
    rng = np.random.default_rng(0)
    thr = []
    cases = [
        (np.array([1, 0, 1, 0, 1]), np.array([0.9, 0.8, 0.7, 0.2, 0.1]), 0.98, 0.6, None, 2.0),
    ]
    for i in range(12):
        n = 20
        y = rng.integers(0, 2, n)
        p = np.clip(rng.normal(0.35 + 0.3 * y, 0.2), 0, 1)
        tr_ = [0.98, 0.9, 0.8, 1.0][i % 4]
        mp = [None, 0.6, 0.9, 0.99][(i // 4) % 4]
        mf = [None, 0.3, 0.05][i % 3]
        cases.append((y, p, tr_, mp, mf, [2.0, 1.0, 0.5][i % 3]))
    cases.append((np.zeros(6, int), np.linspace(0, 1, 6), 0.9, None, None, 2.0))
    for y, p, tr_, mp, mf, fb in cases:
        t, meta = C.select_operating_threshold(y, p, target_recall=tr_, min_precision=mp, max_fpr=mf, f_beta=fb)
        rec_thr = C.find_threshold_for_target_recall(y, p, tr_)
        yp = (p >= t).astype(int)
        conf = C.compute_binary_confusion_metrics(y, yp, 1)
        acc, f1 = C.compute_accuracy_f1(y.tolist(), yp.tolist())
        thr.append({"y": y.tolist(), "p": p.tolist(), "target_recall": tr_, "min_precision": mp, "max_fpr": mf,
                    "f_beta": fb, "threshold": t, "meta": meta, "recall_only_threshold": rec_thr,
                    "confusion_pos1": conf, "acc": acc, "f1": f1})
    goldens["thresholds"] = thr

    # 4. transforms on real dataset images (reference build_transforms / build_transform)
    names = ["avec_labels/cancer/05340cd4-3bb2-459d-9937-bf27d52d8351.jpg",
             "avec_labels/normal/" + sorted(p.name for p in (data / "avec_labels" / "normal").iterdir())[0],
             "sans_label/" + sorted(p.name for p in (data / "sans_label").iterdir())[3]]
    tfs = C.build_transforms(224)
    ext = FE.build_transform()
    srcs, train_out, eval_out, ext_out, flips, angles = [], [], [], [], [], []
    for k, nm in enumerate(names):
        im = Image.open(data / nm).convert("RGB")
        srcs.append(np.asarray(im))
        seed = 100 + k
        torch.manual_seed(seed)
        train_out.append(tfs["train"](im).numpy())
        torch.manual_seed(seed)
        flips.append(bool(torch.rand(1) < 0.5))
        angles.append(float(torch.empty(1).uniform_(-10.0, 10.0).item()))
        eval_out.append(tfs["eval"](im).numpy())
        with Image.open(data / nm) as im2:  # extraction: no convert('RGB') (all RGB)
            ext_out.append(ext(im2).numpy())
    np.savez_compressed(OUT / "transforms.npz", names=np.array(names), src=np.stack(srcs),
                        flip=np.array(flips), angle=np.array(angles), train_out=np.stack(train_out),
                        eval_out=np.stack(eval_out), extract_out=np.stack(ext_out))

    # 5. seeded ResNet-18 (create_model(2, pretrained=False) under seed 42):
    #    logits (eval + train mode) and 512-D embeddings on the transformed images
    torch.manual_seed(42)
    model = C.create_model(2, pretrained=False)
    x = torch.from_numpy(np.stack(eval_out))
    model.eval()
    with torch.no_grad():
        logits_eval = model(x)
        emb = torch.flatten(torch.nn.Sequential(*list(model.children())[:-1])(x), 1)
    model.train()
    with torch.no_grad():
        logits_train = model(x)
    np.savez_compressed(OUT / "resnet18_seed42.npz", x=x.numpy(), logits_eval=logits_eval.numpy(),
                        logits_train=logits_train.numpy(), embeddings=emb.numpy(),
                        running_mean_bn1=model.bn1.running_mean.numpy(), running_var_bn1=model.bn1.running_var.numpy())

    # 6. train_model trajectory (reference loop, tiny synthetic dataset, 3 epochs)
    class Tiny(Dataset):
        def __init__(self, n, seed):
            g = torch.Generator().manual_seed(seed)
            self.x = torch.randn(n, 3, 64, 64, generator=g)
            self.y = torch.tensor([i % 2 for i in range(n)])

        def __len__(self):
            return len(self.y)

        def __getitem__(self, i):
            return self.x[i], int(self.y[i])

    rec6 = _PredRecorder()
    real_metric = C.compute_accuracy_f1
    C.compute_accuracy_f1 = rec6.wrap_metric(real_metric)
    torch.manual_seed(42)
    m2 = C.create_model(2, pretrained=False)
    m2.register_forward_hook(rec6.hook)
    tr_ds, va_ds = Tiny(24, 1), Tiny(8, 2)
    sampler = C.make_balanced_sampler(tr_ds.y.tolist())
    tl = DataLoader(tr_ds, batch_size=8, sampler=sampler, num_workers=0)
    vl = DataLoader(va_ds, batch_size=8, shuffle=False, num_workers=0)
    opt = torch.optim.AdamW((p for p in m2.parameters() if p.requires_grad), lr=1e-4, weight_decay=1e-4)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", patience=2, factor=0.5)
    with tempfile.TemporaryDirectory() as td:
        ck = Path(td) / "best.pt"
        m2, hist = C.train_model(m2, tl, vl, torch.nn.CrossEntropyLoss(), opt, torch.device("cpu"), scheduler=sch,
                                 num_epochs=3, early_stopping_patience=3, model_path=ck)
        saved = torch.load(ck, weights_only=True)
        same = all(torch.equal(saved[k], v) for k, v in m2.state_dict().items())
    C.compute_accuracy_f1 = real_metric
    m2.eval()
    with torch.no_grad():
        final_logits = m2(va_ds.x).numpy()
    goldens["train_model"] = {"history": hist, "final_eval_logits": final_logits.tolist(),
                              "checkpoint_equals_returned": bool(same), "epochs": 3, "batch_size": 8,
                              "metric_calls": rec6.metric_calls}

    # 7. generate_pseudo_labels on fixed logits (identity "model" over a tiny loader)
    class LogitModel(torch.nn.Module):
        def forward(self, z):
            return z

    g = torch.Generator().manual_seed(3)
    z = torch.randn(40, 2, generator=g) * 1.5
    paths = [f"img_{i:03d}.jpg" for i in range(40)]
    pl_loader = DataLoader(list(zip(z, paths)), batch_size=16, shuffle=False)
    pseudo = SS.generate_pseudo_labels(LogitModel(), pl_loader, torch.device("cpu"), threshold=0.7)
    goldens["pseudo_labels"] = {"logits": z.tolist(), "paths": paths, "threshold": 0.7,
                                "selected": [[p, int(l), float(c)] for p, l, c in pseudo]}

    # 8. feature-extraction host helpers on fixed embeddings
    e = np.random.default_rng(5).normal(size=(30, 512)).astype(np.float32)
    recs = [FE.ImageRecord(Path(f"/x/{i}.jpg"), Path(f"sans_label/{i}.jpg"), "unlabeled", None) for i in range(30)]
    goldens["extraction"] = {"embeddings_seed": 5, "shape": [30, 512], "sanity": FE.run_sanity_checks(e),
                             "neighbors": FE.nearest_neighbor_probe(e, recs)}
    recs_ref = FE.discover_image_records(data)
    goldens["extraction"]["records"] = [[str(r.relative_path), r.bucket, r.label] for r in recs_ref]

    # 8b. the schema of the reference's COMMITTED extraction artifacts
    #     (outputs/features/metadata.json, outputs/notes/feature_summary.md)
    meta = json.loads((REF / "outputs/features/metadata.json").read_text())
    summary = (REF / "outputs/notes/feature_summary.md").read_text().splitlines()
    goldens["committed_metadata"] = {
        "keys": list(meta), "sanity_keys": list(meta["sanity_checks"]),
        "probe_keys": list(meta["neighbor_probe"][0]), "embedding_dimension": meta["embedding_dimension"],
        "summary_headings": [ln for ln in summary if ln.startswith("#")],
        "summary_bullets": [ln.split(":")[0] for ln in summary if ln.startswith("- ") and ":" in ln]}

    # 9. the reference's own run_pipeline and run_supervised, end to end on a
    #    tiny deterministic dataset (tests/golden/tiny_dataset.py) with a seeded
    #    stand-in for the ImageNet weights: history, splits, pseudo-labels,
    #    every table / JSON artifact (columns and values)
    goldens["pipeline"] = _pipelines(C, SS)

    # 10. the DataLoader worker stream: (flip, angle) each sample of the train
    #     loader draws inside its worker (num_workers=2), 2 epochs
    goldens["worker_stream"] = _worker_stream(C)

    with open(OUT / "goldens.json", "w") as f:
        json.dump(goldens, f, indent=1, default=float)
    print("wrote", sorted(p.name for p in OUT.iterdir()))


PIPE_CFG = dict(batch_size=4, image_size=64, num_workers=0, baseline_epochs=2, weak_pretrain_epochs=1,
                finetune_epochs=1, pseudo_label_threshold=0.5, target_recall=0.9, min_precision=0.5, seed=42)


def _read_artifacts(out: Path, semi: bool) -> dict:
    import pandas as pd

    def table(p):
        df = pd.read_csv(p, index_col=0)
        if "training_time_sec" in df.columns:  # wall time: not reproducible, kept out of the fixture
            df["training_time_sec"] = None
        return {"columns": list(df.columns), "index": [str(i) for i in df.index],
                "values": json.loads(df.to_json(orient="split"))["data"]}

    art = {"results_comparison": table(out / "tables/results_comparison.csv")}
    if semi:
        art["history"] = json.loads((out / "notes/training_history.json").read_text())
        art["results_comparison_detailed"] = table(out / "tables/results_comparison_detailed.csv")
        art["operating_point"] = json.loads((out / "notes/operating_point.json").read_text())
        tri = pd.read_csv(out / "tables/unlabeled_predictions_semi.csv")
        art["triage"] = {"columns": list(tri.columns), "path": [Path(p).name for p in tri["path"]],
                         "prob_positive": tri["prob_positive"].tolist(), "flagged": tri["flagged"].tolist()}
    art["files"] = sorted(str(p.relative_to(out)) for p in out.rglob("*") if p.is_file())
    return art


def _pipelines(C, SS) -> dict:
    import os

    import torch

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(OUT))
    import tiny_dataset
    from training import supervised as SV  # reference module

    res = {"config": PIPE_CFG, "weights_seed": 1234}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        data = tiny_dataset.make(td / "mri")
        wpath = td / "w.pt"
        torch.save(tiny_dataset.pretrained_state_dict(1234), wpath)
        os.environ["SSIP_RESNET18_WEIGHTS"] = str(wpath)
        picks = []
        real = SS.generate_pseudo_labels

        def spy(*a, **k):
            out = real(*a, **k)
            picks.extend([Path(p).name, int(l), float(c)] for p, l, c in out)
            return out

        real_fns = {(mod, nm): getattr(mod, nm) for mod in (C, SS, SV)
                    for nm in ("create_model", "compute_accuracy_f1", "evaluate_model") if hasattr(mod, nm)}
        try:
            for kind in ("semi", "supervised"):
                rec = _PredRecorder()
                for (mod, nm), fn in real_fns.items():
                    setattr(mod, nm, {"create_model": rec.wrap_create, "compute_accuracy_f1": rec.wrap_metric,
                                      "evaluate_model": rec.wrap_eval}[nm](fn))
                (td / kind).mkdir()
                os.chdir(td / kind)
                cfg = C.TrainingConfig(strong_data_dir=data / "avec_labels", weak_data_dir=data / "sans_label",
                                       device="cpu", **PIPE_CFG)
                if kind == "semi":
                    SS.generate_pseudo_labels = spy
                    metrics = SS.run_pipeline(cfg)
                    SS.generate_pseudo_labels = real
                else:
                    cfg.weak_pretrain_epochs, cfg.finetune_epochs, cfg.pseudo_label_threshold = 0, 0, 0.0
                    metrics = SV.run_supervised(cfg)
                for m in metrics.values():
                    if "training_time_sec" in m:
                        m["training_time_sec"] = None
                res[kind] = {"metrics": json.loads(json.dumps(metrics, default=float)),
                             "artifacts": _read_artifacts(td / kind / "outputs", kind == "semi"),
                             "metric_calls": rec.metric_calls, "eval_calls": rec.eval_calls}
                for (mod, nm), fn in real_fns.items():
                    setattr(mod, nm, fn)
            res["semi"]["pseudo_labels"] = picks
        finally:
            for (mod, nm), fn in real_fns.items():
                setattr(mod, nm, fn)
            os.chdir(cwd)
            os.environ.pop("SSIP_RESNET18_WEIGHTS", None)
            SS.generate_pseudo_labels = real
    return res


REAL_CFG = dict(batch_size=16, image_size=224, num_workers=2, baseline_epochs=10, target_recall=0.98,
                min_precision=0.60, seed=42)
REAL_DIR = OUT / "mri_avec_labels"


def _real_supervised(C) -> None:
    """Section 11: the reference's own run_supervised on the 100 labelled JPEGs
    of mri_dataset_brain_cancer_oc/avec_labels (shipped as fixture data under
    tests/golden/mri_avec_labels/, 2.8 MB, the same file names so the
    ImageFolder order and the stratified split are the reference's) at its
    defaults (batch 16, 224^2, 2 loader workers, 10 baseline epochs, early
    stopping 3) with the threshold policy of its report
    (notes/training_report.md: --target-recall 0.98 --min-precision 0.60),
    the seeded stand-in for the ImageNet weights.  Records every metric and
    evaluate_model call per sample (_PredRecorder) and the history; written to
    tests/golden/real_supervised.json."""
    import os
    import shutil

    import torch

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(OUT))
    import tiny_dataset
    from training import supervised as SV  # reference module

    src = REF / "mri_dataset_brain_cancer_oc" / "avec_labels"
    for cls in ("cancer", "normal"):
        (REAL_DIR / cls).mkdir(parents=True, exist_ok=True)
        for f in sorted((src / cls).iterdir()):
            dst = REAL_DIR / cls / f.name
            if not dst.exists():
                shutil.copyfile(f, dst)
    res = _run_supervised_recorded(C, SV, tiny_dataset)
    # the reference's own run-to-run spread on this set: the same run with
    # torch's CPU convolutions on its non-mkldnn algorithms (another fp32
    # summation order, nothing else changed) -- the yardstick for how far any
    # fp32 implementation's probabilities drift over these AdamW steps
    with torch.backends.mkldnn.flags(enabled=False):
        alt = _run_supervised_recorded(C, SV, tiny_dataset)
    res["alt_no_mkldnn"] = {k: alt[k] for k in ("history", "metric_calls", "eval_calls", "metrics")}
    res.update({"config": REAL_CFG, "weights_seed": 1234, "data": str(src.relative_to(REF))})
    with open(OUT / "real_supervised.json", "w") as f:
        json.dump(res, f, indent=1, default=float)
    print("wrote real_supervised.json:", len(res["metric_calls"]), "metric calls,", len(res["eval_calls"]), "eval calls")


def _run_supervised_recorded(C, SV, tiny_dataset) -> dict:
    import os

    import torch

    cwd = os.getcwd()
    rec = _PredRecorder()
    real_fns = {(mod, nm): getattr(mod, nm) for mod in (C, SV)
                for nm in ("create_model", "compute_accuracy_f1", "evaluate_model") if hasattr(mod, nm)}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        wpath = td / "w.pt"
        torch.save(tiny_dataset.pretrained_state_dict(1234), wpath)
        os.environ["SSIP_RESNET18_WEIGHTS"] = str(wpath)
        hist = {}
        real_train = SV.train_model

        def train_model(*a, **k):
            model, h = real_train(*a, **k)
            hist.update(h)
            return model, h

        try:
            for (mod, nm), fn in real_fns.items():
                setattr(mod, nm, {"create_model": rec.wrap_create, "compute_accuracy_f1": rec.wrap_metric,
                                  "evaluate_model": rec.wrap_eval}[nm](fn))
            SV.train_model = train_model
            os.chdir(td)
            cfg = C.TrainingConfig(strong_data_dir=REAL_DIR, weak_data_dir=REAL_DIR, device="cpu", **REAL_CFG)
            metrics = SV.run_supervised(cfg)
            for m in metrics.values():
                m["training_time_sec"] = None
            art = _read_artifacts(td / "outputs", False)
        finally:
            for (mod, nm), fn in real_fns.items():
                setattr(mod, nm, fn)
            SV.train_model = real_train
            os.chdir(cwd)
            os.environ.pop("SSIP_RESNET18_WEIGHTS", None)
    return {"metrics": json.loads(json.dumps(metrics, default=float)), "artifacts": art,
            "history": json.loads(json.dumps(hist, default=float)),
            "metric_calls": rec.metric_calls, "eval_calls": rec.eval_calls}


class _PredRecorder:
    """Per-sample predictions of the reference run, for prediction-level
    parity: every compute_accuracy_f1 call (the history's
    train_* / val_* values) with the P(class 1) of each of its samples -- the
    softmax of the logits the calling loop took its argmax from, captured by
    a forward hook on every model create_model returns (the last len(y_pred)
    outputs before the call) -- and every evaluate_model call with its
    threshold and per-sample probabilities."""

    def __init__(self):
        self.outs = []
        self.metric_calls = []
        self.eval_calls = []

    def hook(self, _m, _inp, out):
        self.outs.append(out.detach().float().cpu())

    def wrap_create(self, create):
        def create_model(*a, **k):
            m = create(*a, **k)
            m.register_forward_hook(self.hook)
            return m
        return create_model

    def wrap_metric(self, real):
        import torch

        def compute_accuracy_f1(y_true, y_pred):
            n = len(y_pred)
            z = torch.cat(self.outs)[-n:] if n else torch.zeros(0, 2)
            self.outs = []
            p1 = torch.softmax(z, 1)[:, 1]
            assert z.argmax(1).tolist() == list(map(int, y_pred)), "hooked logits do not match the predictions"
            self.metric_calls.append({"y_true": list(map(int, y_true)), "y_pred": list(map(int, y_pred)),
                                      "p1": [float(v) for v in p1]})
            return real(y_true, y_pred)
        return compute_accuracy_f1

    def wrap_eval(self, real):
        def evaluate_model(model, loader, device, pos_index=None, threshold=None):
            out = real(model, loader, device, pos_index=pos_index, threshold=threshold)
            _, yt, yp, pr, _ = out
            self.outs = []
            self.eval_calls.append({"threshold": threshold, "pos_index": pos_index,
                                    "y_true": [int(v) for v in yt], "y_pred": [int(v) for v in yp],
                                    "y_prob": [float(v) for v in pr]})
            return out
        return evaluate_model


class _Recorder:
    """Wraps the reference's train Compose: replays the draws its
    RandomHorizontalFlip / RandomRotation will make (same RNG state, restored)
    and returns them beside the transformed image."""

    def __init__(self, tf):
        self.tf = tf

    def __call__(self, img):
        import torch

        st = torch.get_rng_state()
        flip = bool(torch.rand(1) < 0.5)
        angle = float(torch.empty(1).uniform_(-10.0, 10.0).item())
        torch.set_rng_state(st)
        return self.tf(img), flip, angle


def _worker_stream(C) -> dict:
    import torch

    sys.path.insert(0, str(OUT))
    import tiny_dataset

    with tempfile.TemporaryDirectory() as td:
        data = tiny_dataset.make(Path(td) / "mri", n_per_class=8, n_unl=0, size=40)
        C.set_seed(42)
        tfs = C.build_transforms(32)
        tfs = {"train": _Recorder(tfs["train"]), "eval": tfs["eval"]}
        train_loader, _, _, base, splits = C.prepare_dataloaders(data / "avec_labels", tfs, 3, 0.2, 0.2, 42,
                                                                 num_workers=2)
        epochs = []
        for _ in range(2):
            ep = {"labels": [], "flip": [], "angle": []}
            for (img, flips, angles), labels in train_loader:
                ep["labels"] += labels.tolist()
                ep["flip"] += [bool(f) for f in flips]
                ep["angle"] += [float(a) for a in angles]
            epochs.append(ep)
    return {"n_per_class": 8, "size": 40, "image_size": 32, "batch_size": 3, "num_workers": 2, "seed": 42,
            "train_idx": splits["train"].tolist(), "epochs": epochs}


if __name__ == "__main__":
    main()
