"""Feature extraction (512-D global-average-pool embeddings) — drop-in mirror
of the reference's src/feature_extraction.py with the compute on the HIP
kernels.

Same CLI (--data-dir, --device, --batch-size, --verbose; :510-535), same
record discovery order (:125-181), same transform semantics (Resize(256) ->
CenterCrop(224) -> ToTensor -> Normalize, :184-207; executed Pillow-exactly
on the GPU), same artifacts under outputs/ (:401-502): embeddings.npy (f32
[N,512]), embeddings.csv, metadata.json, logs/feature_extraction.log,
notes/feature_summary.md.  Decode failures are logged and skipped (:276-284).
JPEG decode runs on a host thread pool (PIL releases the GIL) instead of
sequentially in the main process.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import logging
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from datetime import datetime, timezone
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch
from PIL import Image, UnidentifiedImageError

_PKG = Path(__file__).resolve().parents[1]
if str(_PKG) not in sys.path:
    sys.path.insert(0, str(_PKG))

from ssip.dist import shard_range  # noqa: E402
from .training import distributed as D  # noqa: E402
from ssip import SSIPResNet  # noqa: E402
from ssip.augment import GpuTransform  # noqa: E402
from ssip.host import pil_extraction_transform  # noqa: E402

DEFAULT_DATA_DIR = Path("mri_dataset_brain_cancer_oc")
DEFAULT_OUTPUT_ROOT = Path("outputs")
FEATURE_OUTPUT_DIR = DEFAULT_OUTPUT_ROOT / "features"
LOG_OUTPUT_DIR = DEFAULT_OUTPUT_ROOT / "logs"
NOTE_OUTPUT_DIR = DEFAULT_OUTPUT_ROOT / "notes"
LOG_PATH = LOG_OUTPUT_DIR / "feature_extraction.log"
EMBEDDING_ARRAY_PATH = FEATURE_OUTPUT_DIR / "embeddings.npy"
EMBEDDING_CSV_PATH = FEATURE_OUTPUT_DIR / "embeddings.csv"
METADATA_PATH = FEATURE_OUTPUT_DIR / "metadata.json"
SUMMARY_NOTE_PATH = NOTE_OUTPUT_DIR / "feature_summary.md"

IMAGENET_MEAN = [0.485, 0.456, 0.406]
IMAGENET_STD = [0.229, 0.224, 0.225]
TARGET_RESIZE = 256
TARGET_CROP = 224
BATCH_SIZE = 32
NEIGHBOR_SAMPLE = 8
RNG_SEED = 42

LABELED_BUCKET = "avec_labels"
UNLABELED_BUCKET = "sans_label"

BACKBONE_NAME = "torchvision.resnet18"
BACKBONE_WEIGHTS = "ResNet18_Weights.IMAGENET1K_V1"
BACKBONE_LAYER = "global_avg_pool"
WEIGHTS_ENV = "SSIP_RESNET18_WEIGHTS"


@dataclass(frozen=True)
class ImageRecord:
    absolute_path: Path
    relative_path: Path
    bucket: str
    label: Optional[str]


@dataclass
class ExtractionResults:
    embeddings: np.ndarray
    records: List[ImageRecord]
    failures: List[Path]
    per_file_times: List[float]
    weights: str = BACKBONE_WEIGHTS   # what the backbone was initialised from (metadata.json "weights")


def configure_logging(verbose: bool = False) -> None:
    LOG_OUTPUT_DIR.mkdir(parents=True, exist_ok=True)
    logging.basicConfig(level=logging.DEBUG if verbose else logging.INFO,
                        format="%(asctime)s [%(levelname)s] %(message)s",
                        handlers=[logging.FileHandler(LOG_PATH, mode="w", encoding="utf-8"), logging.StreamHandler()])


def discover_image_records(data_dir: Path) -> List[ImageRecord]:
    """Labelled folders (sorted) then the flat unlabelled bucket, files sorted."""
    if not data_dir.exists():
        raise FileNotFoundError(f"Data directory not found: {data_dir}")
    records: List[ImageRecord] = []
    lab = data_dir / LABELED_BUCKET
    if lab.exists():
        for d in sorted(p for p in lab.iterdir() if p.is_dir()):
            for f in sorted(d.rglob("*")):
                if f.is_file():
                    records.append(ImageRecord(f, f.relative_to(data_dir), "labeled", d.name))
    else:
        logging.warning("Labeled bucket missing at %s", lab)
    unl = data_dir / UNLABELED_BUCKET
    if unl.exists():
        for f in sorted(unl.rglob("*")):
            if f.is_file():
                records.append(ImageRecord(f, f.relative_to(data_dir), "unlabeled", None))
    else:
        logging.warning("Unlabeled bucket missing at %s", unl)
    if not records:
        raise RuntimeError(f"No image files discovered under {data_dir}")
    logging.info("Discovered %d images (labeled=%d, unlabeled=%d)", len(records),
                 sum(r.bucket == "labeled" for r in records), sum(r.bucket == "unlabeled" for r in records))
    return records


def build_transform(dtype: torch.dtype = torch.float32) -> GpuTransform:
    """Resize(256) (short side) -> CenterCrop(224) -> ToTensor -> Normalize, on the device."""
    return GpuTransform(dtype=dtype, mode="short", resize=TARGET_RESIZE, crop=TARGET_CROP, mean=IMAGENET_MEAN,
                        std=IMAGENET_STD)


def load_model(device: torch.device, dtype: str = "fp32", weights: Optional[Path] = None,
               allow_random_init: bool = False) -> SSIPResNet:
    """Frozen eval-mode ResNet-18 returning the [B,512,1,1] avgpool output
    (the reference's nn.Sequential(children()[:-1]), feature_extraction.py:210-227).
    The IMAGENET1K_V1 download of the reference is a local state_dict here
    (`weights` / $SSIP_RESNET18_WEIGHTS); without one this raises, as the
    reference's failed download does, unless the seeded random backbone was
    opted in to (--random-init / $SSIP_ALLOW_RANDOM_INIT=1); metadata.json's
    "weights" then says so."""
    import os

    path = weights or os.environ.get(WEIGHTS_ENV)
    torch.manual_seed(RNG_SEED)
    model = SSIPResNet("resnet18", num_classes=1000, dtype=dtype)
    if path and Path(path).exists():
        model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        model.init_source = BACKBONE_WEIGHTS
    elif allow_random_init or os.environ.get("SSIP_ALLOW_RANDOM_INIT") == "1":
        logging.warning("%s unavailable offline; embeddings use the seeded (seed %d) random initialisation "
                        "(opted in)", BACKBONE_WEIGHTS, RNG_SEED)
        model.init_source = f"random_init(seed={RNG_SEED})"
    else:
        raise RuntimeError(f"{BACKBONE_WEIGHTS} is a network download and no local copy was given: pass --weights "
                           f"<torchvision resnet18 state_dict> or set {WEIGHTS_ENV}, or opt in to the seeded random "
                           "backbone with --random-init (or SSIP_ALLOW_RANDOM_INIT=1)")
    model.eval()
    for p in model.parameters():
        p.requires_grad_(False)
    model.embedding_only = True
    # --device cpu (BASELINE config 1, the reference's feature_extraction.py:
    # 519-522,542): the same module tree evaluated with torch's CPU operators
    model.host_execution = device.type == "cpu"
    return model.to(device)


def _as_rgb(img: Image.Image) -> Image.Image:
    """The reference does not convert (its inputs are RGB: feature_extraction.py
    :232-240), and its Normalize raises on any other mode.  Both device paths
    here take Pillow's RGB conversion instead (grayscale replicated, alpha
    dropped, palettes expanded), so the HIP and --device cpu paths see the
    same pixels for every file; an RGB file is passed through untouched."""
    return img if img.mode == "RGB" else img.convert("RGB")


def preprocess_image(path: Path) -> np.ndarray:
    """Decode to uint8 [H, W, 3] (RGB files as they are, others via _as_rgb)."""
    with Image.open(path) as img:
        a = np.asarray(_as_rgb(img))
    return np.ascontiguousarray(a)


def batched(items: Sequence, batch_size: int) -> Iterable[Sequence]:
    for s in range(0, len(items), batch_size):
        yield items[s:min(s + batch_size, len(items))]


def extract_embeddings(records: List[ImageRecord], device: torch.device, batch_size: int = BATCH_SIZE,
                       dtype: str = "fp32", weights: Optional[Path] = None,
                       decode_threads: int = 8, allow_random_init: bool = False) -> ExtractionResults:
    if device.type == "cpu":
        # the host path is the reference's fp32 loop on one process
        if dtype != "fp32":
            raise RuntimeError("extract_embeddings: --device cpu computes in fp32 (the reference's precision), "
                               f"not {dtype}")
        if D.world() > 1:
            raise RuntimeError("extract_embeddings: --device cpu runs in one process (torchrun shards the HIP "
                               "path only: every rank would extract every file and write the same outputs)")
        return _extract_embeddings_host(records, batch_size, weights, decode_threads, allow_random_init)
    model = load_model(device, dtype, weights, allow_random_init)
    tf = build_transform(model.compute_dtype)
    embeddings: List[np.ndarray] = []
    kept: List[ImageRecord] = []
    failures: List[Path] = []
    times: List[float] = []
    logging.info("Beginning feature extraction over %d records", len(records))

    def decode(rec):
        try:
            return rec, preprocess_image(rec.absolute_path), None
        except (UnidentifiedImageError, OSError) as exc:
            return rec, None, exc

    # data parallel (torchrun): this rank's contiguous run of whole batches; the
    # per-batch results are gathered in rank order = the single-process order
    mine = records
    if D.world() > 1:
        nb = (len(records) + batch_size - 1) // batch_size
        blo, bhi = shard_range(nb, D.rank(), D.world())
        mine = records[blo * batch_size:min(bhi * batch_size, len(records))]
    chunks = list(batched(mine, batch_size))
    with ThreadPoolExecutor(max_workers=decode_threads) as pool:
        # decode runs PREFETCH batches ahead of the device (Pillow releases the
        # GIL while decoding); embeddings stay on the device until the end, so
        # the loop never waits for the GPU
        PREFETCH = 2
        pending = [[pool.submit(decode, r) for r in c] for c in chunks[:PREFETCH]]
        t_prev = time.perf_counter()
        for ci in range(len(chunks)):
            if ci + PREFETCH < len(chunks):
                pending.append([pool.submit(decode, r) for r in chunks[ci + PREFETCH]])
            ok_recs, arrays = [], []
            for fut in pending[ci]:
                rec, arr, exc = fut.result()
                if exc is not None:
                    logging.error("Failed to decode %s: %s", rec.absolute_path, exc)
                    failures.append(rec.absolute_path)
                    continue
                ok_recs.append(rec)
                arrays.append(arr)
            pending[ci] = None
            if not arrays:
                continue
            with torch.no_grad():
                if len({a.shape for a in arrays}) == 1:
                    u8 = torch.from_numpy(np.stack(arrays)).pin_memory().to(device, non_blocking=True)
                    feats = model(tf(u8)).flatten(1)
                else:
                    feats = torch.cat([model(tf(torch.from_numpy(a)[None].to(device))).flatten(1) for a in arrays])
            embeddings.append(feats)
            kept.extend(ok_recs)
            t_now = time.perf_counter()
            times.extend([(t_now - t_prev) / len(ok_recs)] * len(ok_recs))
            t_prev = t_now
    embeddings = [torch.cat(embeddings).cpu().numpy()] if embeddings else []
    if D.world() > 1:
        embeddings, kept, failures, times = (D.gather_list(v) for v in (embeddings, kept, failures, times))
    if not embeddings:
        raise RuntimeError("No embeddings were generated; all images failed to decode?")
    mat = np.concatenate(embeddings, 0)
    logging.info("Computed embeddings with shape %s", mat.shape)
    return ExtractionResults(mat, kept, failures, times, model.init_source)


def _extract_embeddings_host(records: List[ImageRecord], batch_size: int, weights: Optional[Path],
                             decode_threads: int, allow_random_init: bool) -> ExtractionResults:
    """--device cpu: the reference's loop (decode + transform per file, a
    stacked batch through the frozen backbone, fp32), with the per-file
    decode + transform on a host thread pool (ssip/host.py)."""
    model = load_model(torch.device("cpu"), "fp32", weights, allow_random_init)
    embeddings: List[np.ndarray] = []
    kept: List[ImageRecord] = []
    failures: List[Path] = []
    times: List[float] = []
    logging.info("Beginning feature extraction over %d records (host)", len(records))

    def load(rec):
        try:
            with Image.open(rec.absolute_path) as img:
                return rec, pil_extraction_transform(_as_rgb(img), TARGET_RESIZE, TARGET_CROP, IMAGENET_MEAN,
                                                     IMAGENET_STD), None
        except (UnidentifiedImageError, OSError) as exc:
            return rec, None, exc

    with ThreadPoolExecutor(max_workers=decode_threads) as pool:
        for chunk in batched(records, batch_size):
            t0 = time.perf_counter()
            ok_recs, tensors = [], []
            for rec, t, exc in pool.map(load, chunk):
                if exc is not None:
                    logging.error("Failed to decode %s: %s", rec.absolute_path, exc)
                    failures.append(rec.absolute_path)
                    continue
                ok_recs.append(rec)
                tensors.append(t)
            if not tensors:
                continue
            with torch.no_grad():
                feats = model(torch.stack(tensors)).flatten(1)
            embeddings.append(feats.numpy())
            kept.extend(ok_recs)
            per = (time.perf_counter() - t0) / len(ok_recs)
            times.extend([per] * len(ok_recs))
    if not embeddings:
        raise RuntimeError("No embeddings were generated; all images failed to decode?")
    mat = np.concatenate(embeddings, 0)
    logging.info("Computed embeddings with shape %s", mat.shape)
    return ExtractionResults(mat, kept, failures, times, model.init_source)


def compute_dataset_digest(records: Sequence[ImageRecord]) -> str:
    h = hashlib.sha256()
    for r in sorted(records, key=lambda r: str(r.relative_path)):
        st = r.absolute_path.stat()
        h.update(str(r.relative_path).encode("utf-8"))
        h.update(str(st.st_size).encode("utf-8"))
        h.update(str(int(st.st_mtime)).encode("utf-8"))
    return h.hexdigest()


def run_sanity_checks(embeddings: np.ndarray) -> Dict[str, float]:
    if np.isnan(embeddings).any():
        raise ValueError("Embedding matrix contains NaN values")
    if np.isinf(embeddings).any():
        raise ValueError("Embedding matrix contains inf values")
    stats = {"num_vectors": int(embeddings.shape[0]), "dimension": int(embeddings.shape[1]),
             "mean_abs_mean": float(np.abs(embeddings.mean(axis=0)).mean()),
             "mean_std": float(embeddings.std(axis=0).mean())}
    logging.info("Embedding stats — vectors: %d, dim: %d, mean(|mean|): %.5f, mean(std): %.5f",
                 stats["num_vectors"], stats["dimension"], stats["mean_abs_mean"], stats["mean_std"])
    return stats


def nearest_neighbor_probe(embeddings: np.ndarray, records: Sequence[ImageRecord], sample_size: int = NEIGHBOR_SAMPLE,
                           seed: int = RNG_SEED) -> List[Dict[str, object]]:
    if embeddings.shape[0] < 2:
        return []
    rng = np.random.default_rng(seed)
    sample_size = min(sample_size, embeddings.shape[0] - 1)
    if sample_size <= 0:
        return []
    picks = rng.choice(embeddings.shape[0], size=sample_size, replace=False)
    norms = np.clip(np.linalg.norm(embeddings, axis=1, keepdims=True), 1e-12, None)
    unit = embeddings / norms
    out = []
    for i in picks:
        sims = unit[i] @ unit.T
        sims[i] = -np.inf
        j = int(np.argmax(sims))
        out.append({"query": str(records[i].relative_path), "neighbor": str(records[j].relative_path),
                    "similarity": float(sims[j])})
    logging.info("Nearest-neighbor probe completed for %d samples", len(out))
    return out


def save_artifacts(results: ExtractionResults, stats: Dict[str, float], probe: List[Dict[str, object]],
                   data_dir: Path, device: torch.device) -> None:
    import pandas as pd

    FEATURE_OUTPUT_DIR.mkdir(parents=True, exist_ok=True)
    NOTE_OUTPUT_DIR.mkdir(parents=True, exist_ok=True)
    np.save(EMBEDDING_ARRAY_PATH, results.embeddings.astype(np.float32))
    pd.DataFrame([{"index": i, "path": str(r.relative_path), "bucket": r.bucket, "label": r.label}
                  for i, r in enumerate(results.records)]).to_csv(EMBEDDING_CSV_PATH, index=False)
    meta = {"backbone": BACKBONE_NAME, "weights": results.weights, "layer": BACKBONE_LAYER,
            "embedding_dimension": int(results.embeddings.shape[1]), "input_resize": TARGET_RESIZE,
            "input_crop": TARGET_CROP, "normalization_mean": IMAGENET_MEAN, "normalization_std": IMAGENET_STD,
            "channel_policy": "No conversion (assumes RGB inputs)",
            "date_utc": datetime.now(timezone.utc).isoformat(), "num_images": int(results.embeddings.shape[0]),
            "failed_images": len(results.failures), "device": str(device), "dataset_dir": str(data_dir),
            "dataset_digest": compute_dataset_digest(results.records), "sanity_checks": stats,
            "neighbor_probe": probe}
    with METADATA_PATH.open("w", encoding="utf-8") as f:
        json.dump(meta, f, indent=2)
    fails = "None" if not results.failures else "\n".join(f"- {p}" for p in results.failures)
    mean_l = float(np.mean(results.per_file_times)) if results.per_file_times else float("nan")
    med_l = float(np.median(results.per_file_times)) if results.per_file_times else float("nan")
    lines = ["| Query | Neighbor | Cosine |", "| --- | --- | --- |"]
    lines += [f"| {it['query']} | {it['neighbor']} | {it['similarity']:.4f} |" for it in probe]
    nb = "\n".join(lines) if probe else "No neighbors computed (insufficient samples)."
    SUMMARY_NOTE_PATH.write_text(f"""# Feature Extraction Summary

- Backbone: {BACKBONE_NAME} ({results.weights})
- Layer: global average pooled features ({results.embeddings.shape[1]}-D)
- Input spec: resize {TARGET_RESIZE} → center crop {TARGET_CROP}, ImageNet normalization
- Batch size: {BATCH_SIZE}
- Device: {device}
- Total images processed: {results.embeddings.shape[0]}
- Failed decodes: {len(results.failures)}
- Mean per-image latency (s): {mean_l:.4f}
- Median per-image latency (s): {med_l:.4f}

## Sanity Check Statistics

- Mean of |dimension means|: {stats['mean_abs_mean']:.6f}
- Mean of dimension standard deviations: {stats['mean_std']:.6f}

## Nearest Neighbor Spot Check

{nb}

## Decode Failures

{fails}
""", encoding="utf-8")


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="Extract CNN embeddings for the MRI dataset")
    p.add_argument("--data-dir", type=Path, default=DEFAULT_DATA_DIR,
                   help="Root directory containing 'avec_labels' and 'sans_label'")
    p.add_argument("--device", type=str, default="cuda" if torch.cuda.is_available() else "cpu",
                   help="Torch device to use (default: cuda if available else cpu)")
    p.add_argument("--batch-size", type=int, default=BATCH_SIZE, help="Mini-batch size for inference")
    p.add_argument("--verbose", action="store_true", help="Enable verbose logging")
    p.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--weights", type=Path, default=None)
    p.add_argument("--random-init", action="store_true",
                   help="Allow the seeded random backbone when no ImageNet weights are available locally")
    return p.parse_args(argv)


def main(argv=None) -> None:
    args = parse_args(argv)
    configure_logging(verbose=args.verbose)
    device = torch.device(args.device)
    if device.type not in ("cuda", "cpu"):
        raise RuntimeError(f"ssip feature extraction runs on the HIP device (--device cuda) or the host "
                           f"(--device cpu), not {device}")
    if device.type == "cuda":
        device = D.setup(device)  # torchrun: one rank per GPU, file list sharded by batch
    elif args.dtype != "fp32":
        raise RuntimeError("--device cpu computes in fp32 (the reference's precision)")
    logging.info("Starting feature extraction on device %s", device)
    records = discover_image_records(args.data_dir)
    t0 = time.perf_counter()
    res = extract_embeddings(records, device=device, batch_size=args.batch_size, dtype=args.dtype,
                             weights=args.weights, allow_random_init=args.random_init)
    logging.info("Completed embedding extraction in %.2f seconds", time.perf_counter() - t0)
    stats = run_sanity_checks(res.embeddings)
    probe = nearest_neighbor_probe(res.embeddings, res.records)
    if D.is_main():
        save_artifacts(res, stats, probe, args.data_dir, device)
        logging.info("Artifacts saved to %s", FEATURE_OUTPUT_DIR)


if __name__ == "__main__":
    main()
