"""`python -m src.feature_extraction --device cpu` (BASELINE config 1; the
reference's feature_extraction.py:519-522,542): the product's own module
tree and transform on the host (ssip/host.py), checked against the goldens
the reference's own code produced (tests/golden/make_goldens.py) -- the
transform bit for bit (the same Pillow calls), embeddings / logits rel-max
1e-5 -- and, on a GPU box, against the HIP fp32 extraction of the same files
(rel-max 1e-5 per the north star's fp32 tolerance).  No oracle import."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch
from PIL import Image

GOLD_DIR = Path(__file__).parent / "golden"


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def _dataset(root: Path, n_per_class=4, n_unl=6, size=96):
    rng = np.random.default_rng(0)
    for cls, bias in (("cancer", 60), ("normal", 180)):
        d = root / "avec_labels" / cls
        d.mkdir(parents=True)
        for i in range(n_per_class):
            a = np.clip(rng.normal(bias, 40, (size, size + 16 * i, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(a).save(d / f"{cls}_{i:02d}.jpg", quality=90)
    u = root / "sans_label"
    u.mkdir(parents=True)
    for i in range(n_unl):
        a = np.clip(rng.normal(120, 50, (size + 8 * i, size, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(a).save(u / f"u_{i:03d}.jpg", quality=90)
    (u / "broken.jpg").write_bytes(b"not a jpeg")  # a decode failure is logged and skipped
    # non-RGB files: grayscale, RGBA and palette PNGs take Pillow's
    # RGB conversion on both device paths
    g = np.clip(rng.normal(110, 40, (size, size + 8)), 0, 255).astype(np.uint8)
    Image.fromarray(g, "L").save(u / "v_gray.png")
    rgba = np.clip(rng.normal(140, 40, (size + 4, size, 4)), 0, 255).astype(np.uint8)
    Image.fromarray(rgba, "RGBA").save(u / "v_rgba.png")
    Image.fromarray(np.clip(rng.normal(100, 60, (size, size, 3)), 0, 255).astype(np.uint8)).quantize(16).save(
        u / "v_pal.png")
    return root


def test_host_transform_matches_reference_golden():
    from src import feature_extraction as FE
    from ssip.host import pil_extraction_transform

    g = np.load(GOLD_DIR / "transforms.npz")
    for src, want in zip(g["src"], g["extract_out"]):
        got = pil_extraction_transform(Image.fromarray(src), FE.TARGET_RESIZE, FE.TARGET_CROP, FE.IMAGENET_MEAN,
                                       FE.IMAGENET_STD)
        assert np.array_equal(got.numpy(), want)


def test_host_forward_matches_reference_golden():
    from src import feature_extraction as FE

    g = np.load(GOLD_DIR / "resnet18_seed42.npz")
    m = FE.load_model(torch.device("cpu"), "fp32", None, allow_random_init=True)
    x = torch.from_numpy(g["x"])
    emb = m(x).flatten(1).numpy()
    assert _rel(emb, g["embeddings"]) < 1e-5
    # the SSIPResNet parameter container raises on the CPU unless asked for
    m.host_execution = False
    with pytest.raises(RuntimeError, match="HIP device"):
        m(x)


def test_cli_device_cpu(tmp_path, monkeypatch):
    data = _dataset(tmp_path / "mri")
    monkeypatch.chdir(tmp_path)
    from src import feature_extraction as FE

    FE.main(["--data-dir", str(data), "--device", "cpu", "--batch-size", "32", "--random-init"])
    emb = np.load(tmp_path / "outputs/features/embeddings.npy")
    assert emb.shape == (17, 512) and emb.dtype == np.float32 and np.isfinite(emb).all()
    meta = json.loads((tmp_path / "outputs/features/metadata.json").read_text())
    gm = json.loads((GOLD_DIR / "goldens.json").read_text())["committed_metadata"]
    assert meta["device"] == "cpu" and meta["num_images"] == 17 and meta["failed_images"] == 1
    for k in gm["keys"]:
        assert k in meta, k
    for f in ("features/embeddings.csv", "logs/feature_extraction.log", "notes/feature_summary.md"):
        assert (tmp_path / "outputs" / f).exists(), f


def test_non_rgb_inputs_take_the_rgb_conversion(tmp_path):
    """Both device paths decode through the same RGB conversion: the HIP
    path's uint8 input is Pillow's convert('RGB') of every non-RGB file."""
    from src import feature_extraction as FE

    data = _dataset(tmp_path / "mri", n_per_class=1, n_unl=1)
    for nm in ("v_gray.png", "v_rgba.png", "v_pal.png"):
        f = data / "sans_label" / nm
        with Image.open(f) as im:
            assert im.mode != "RGB"
            want = np.asarray(im.convert("RGB"))
        got = FE.preprocess_image(f)
        assert got.shape == want.shape and got.dtype == np.uint8 and np.array_equal(got, want), nm


def test_host_path_refuses_bf16_and_world(monkeypatch, tmp_path):
    from src import feature_extraction as FE
    from src.training import distributed as D

    recs = FE.discover_image_records(_dataset(tmp_path / "mri", n_per_class=1, n_unl=1))
    with pytest.raises(RuntimeError, match="fp32"):
        FE.extract_embeddings(recs, torch.device("cpu"), dtype="bf16", allow_random_init=True)
    monkeypatch.setattr(D, "world", lambda: 2)
    with pytest.raises(RuntimeError, match="one process"):
        FE.extract_embeddings(recs, torch.device("cpu"), allow_random_init=True)


@pytest.mark.gpu
def test_host_extraction_matches_hip_fp32(dev, tmp_path):
    from src import feature_extraction as FE

    data = _dataset(tmp_path / "mri")
    recs = FE.discover_image_records(data)
    cpu = FE.extract_embeddings(recs, torch.device("cpu"), batch_size=32, allow_random_init=True)
    hip = FE.extract_embeddings(recs, dev, batch_size=32, dtype="fp32", allow_random_init=True)
    assert [r.relative_path for r in cpu.records] == [r.relative_path for r in hip.records]
    assert len(cpu.failures) == len(hip.failures) == 1
    assert _rel(cpu.embeddings, hip.embeddings) < 1e-5
