"""CPU: host-side logic of the drop-in pipeline vs golden vectors generated
from the reference's own code (tests/golden/make_goldens.py): split
indices (bit-exact), balanced sampler weights + draws (bit-exact),
threshold selection / confusion metrics, extraction helpers, record
discovery order."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

GOLD = json.loads((Path(__file__).parent / "golden" / "goldens.json").read_text())


@pytest.fixture(scope="module")
def C():
    from src.training import common

    return common


def test_split_real_dataset_bit_exact(C):
    g = GOLD["splits"]
    for seed, exp in g["by_seed"].items():
        tr, va, te = C.stratified_split(g["targets"], 0.2, 0.2, int(seed))
        assert tr.tolist() == exp["train"] and va.tolist() == exp["val"] and te.tolist() == exp["test"]
    s = g["synthetic"]
    tr, va, te = C.stratified_split(s["targets"], s["val"], s["test"], s["seed"])
    assert tr.tolist() == s["train"] and va.tolist() == s["val_idx"] and te.tolist() == s["test_idx"]


def test_survey_appendix_c_split(C):
    tr, va, te = C.stratified_split([0] * 50 + [1] * 50, 0.2, 0.2, 42)
    assert tr[:5].tolist() == [74, 33, 88, 5, 9] and va[:3].tolist() == [53, 49, 20] and te[-2:].tolist() == [40, 75]


def test_balanced_sampler(C):
    for case in GOLD["sampler"]:
        s = C.make_balanced_sampler(case["labels"])
        assert s.num_samples == case["num_samples"]
        assert np.allclose(s.weights.numpy(), case["weights"], rtol=0, atol=0)
        torch.manual_seed(case["seed"])
        assert [int(i) for i in iter(s)] == case["draws"]


def test_threshold_selection(C):
    for c in GOLD["thresholds"]:
        y, p = np.array(c["y"]), np.array(c["p"])
        t, meta = C.select_operating_threshold(y, p, target_recall=c["target_recall"], min_precision=c["min_precision"],
                                               max_fpr=c["max_fpr"], f_beta=c["f_beta"])
        assert t == c["threshold"]
        assert meta == c["meta"]
        assert C.find_threshold_for_target_recall(y, p, c["target_recall"]) == c["recall_only_threshold"]
        yp = (p >= t).astype(int)
        assert C.compute_binary_confusion_metrics(y, yp, 1) == c["confusion_pos1"]
        acc, f1 = C.compute_accuracy_f1(y.tolist(), yp.tolist())
        assert acc == c["acc"] and f1 == c["f1"]


def test_extraction_helpers():
    from src import feature_extraction as FE

    e = np.random.default_rng(GOLD["extraction"]["embeddings_seed"]).normal(size=tuple(GOLD["extraction"]["shape"]))
    e = e.astype(np.float32)
    assert FE.run_sanity_checks(e) == GOLD["extraction"]["sanity"]
    recs = [FE.ImageRecord(Path(f"/x/{i}.jpg"), Path(f"sans_label/{i}.jpg"), "unlabeled", None) for i in range(30)]
    got = FE.nearest_neighbor_probe(e, recs)
    exp = GOLD["extraction"]["neighbors"]
    assert [(g["query"], g["neighbor"]) for g in got] == [(x["query"], x["neighbor"]) for x in exp]
    assert np.allclose([g["similarity"] for g in got], [x["similarity"] for x in exp], rtol=1e-6)


def test_discovery_order_and_imagefolder(tmp_path):
    """Rebuild the dataset's file tree (empty files) and check the
    discovery order of both the ImageFolder and the extraction records."""
    from src import feature_extraction as FE
    from ssip.data import ImageFolder

    root = tmp_path / "mri"
    for rel, _, _ in GOLD["extraction"]["records"]:
        f = root / rel
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_bytes(b"")
    recs = FE.discover_image_records(root)
    assert [[str(r.relative_path), r.bucket, r.label] for r in recs] == GOLD["extraction"]["records"]
    ds = ImageFolder(root / "avec_labels")
    assert ds.classes == GOLD["splits"]["classes"]
    assert [str(Path(p).relative_to(root)) for p, _ in ds.samples] == GOLD["splits"]["samples"]
    assert ds.targets == GOLD["splits"]["targets"]


def test_cli_surface():
    from src import semi_supervised_training as S
    from src import supervised_training as T

    c = S.parse_args(["--strong-data-dir", "a", "--weak-data-dir", "b"])
    assert (c.batch_size, c.val_split, c.test_split, c.seed, c.image_size, c.num_workers) == (16, 0.2, 0.2, 42, 224, 2)
    assert (c.baseline_epochs, c.weak_pretrain_epochs, c.finetune_epochs, c.pseudo_label_threshold) == (10, 5, 8, 0.7)
    assert (c.learning_rate, c.weight_decay, c.early_stopping_patience, c.positive_class) == (1e-4, 1e-4, 3, "cancer")
    assert c.device == "auto" and str(c.semi_checkpoint) == "outputs/models/semi_resnet18.pt"
    t = T.parse_args(["--strong-data-dir", "a", "--output-dir", "o"])
    assert str(t.weak_data_dir) == "unused" and t.weak_pretrain_epochs == 0 and t.pseudo_label_threshold == 0.0
    assert str(t.baseline_checkpoint) == "o/models/baseline_resnet18.pt"
    with pytest.raises(SystemExit):
        S.parse_args(["--strong-data-dir", "a"])  # --weak-data-dir is required for the semi CLI


def test_transform_spec_rng_matches_torchvision_order():
    """The worker-side spec draws flip then angle with torchvision's calls."""
    from PIL import Image

    from src.training.common import build_transforms

    spec = build_transforms(224)["train"]
    img = Image.fromarray(np.zeros((512, 512, 3), np.uint8))
    torch.manual_seed(7)
    h = spec(img)
    torch.manual_seed(7)
    flip = bool(torch.rand(1) < 0.5)
    angle = float(torch.empty(1).uniform_(-10.0, 10.0).item())
    from ssip.augment import rotate_fixed_point

    assert int(h.params[0]) == int(flip) and int(h.params[1]) == 1
    assert tuple(int(v) for v in h.params[2:8]) == rotate_fixed_point(angle, 224, 224)


def test_create_model_without_weights_raises_unless_opted_in(monkeypatch):
    """The reference's create_model downloads IMAGENET1K_V1 or fails
    (common.py:299-304); offline, pretrained=True must fail the same way
    unless the seeded random backbone is explicitly requested."""
    from src.training.common import create_model

    monkeypatch.delenv("SSIP_RESNET18_WEIGHTS", raising=False)
    monkeypatch.delenv("SSIP_ALLOW_RANDOM_INIT", raising=False)
    with pytest.raises(RuntimeError, match="random-init"):
        create_model(2, pretrained=True)
    m = create_model(2, pretrained=True, allow_random_init=True)
    assert m.init_source == "random_init"
    monkeypatch.setenv("SSIP_ALLOW_RANDOM_INIT", "1")
    assert create_model(2, pretrained=True).init_source == "random_init"
    assert create_model(2, pretrained=False).fc.out_features == 2


def test_cli_random_init_flag():
    from src import feature_extraction as FE
    from src import semi_supervised_training as S

    assert S.parse_args(["--strong-data-dir", "a", "--weak-data-dir", "b"]).random_init is False
    assert S.parse_args(["--strong-data-dir", "a", "--weak-data-dir", "b", "--random-init"]).random_init is True
    assert FE.parse_args(["--random-init"]).random_init is True


def test_dataloader_worker_stream_matches_reference(tmp_path):
    """The (flip, angle) each train sample draws inside its DataLoader worker
    (num_workers=2, 2 epochs: worker w seeded base_seed + w, base_seed and the
    balanced sampler's multinomial from the global RNG each epoch) equals the
    reference's own loader's draws (tests/golden: the reference's
    prepare_dataloaders with a recording wrapper around its train Compose)."""
    import sys

    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    import tiny_dataset
    from src.training import common as C
    from ssip.augment import rotate_fixed_point

    ws = GOLD["worker_stream"]
    data = tiny_dataset.make(tmp_path / "mri", n_per_class=ws["n_per_class"], n_unl=0, size=ws["size"])
    C.set_seed(ws["seed"])
    tfs = C.build_transforms(ws["image_size"])
    train_loader, _, _, _, splits = C.prepare_dataloaders(data / "avec_labels", tfs, ws["batch_size"], 0.2, 0.2,
                                                          ws["seed"], num_workers=ws["num_workers"])
    assert splits["train"].tolist() == ws["train_idx"]
    S = ws["image_size"]
    for ep in ws["epochs"]:
        labels, params = [], []
        for batch, lab in train_loader:
            labels += lab.tolist()
            params.append(batch.params)
        p = torch.cat(params)
        assert labels == ep["labels"]
        assert [bool(f) for f in p[:, 0]] == ep["flip"]
        for row, ang in zip(p.tolist(), ep["angle"]):
            assert tuple(row[2:8]) == rotate_fixed_point(ang, S, S)


def test_extraction_artifact_schema_matches_committed(tmp_path, monkeypatch):
    """metadata.json (keys and their order, sanity / neighbour-probe sub-keys)
    and feature_summary.md (headings, bullet labels) as the reference's
    committed outputs/features/metadata.json and outputs/notes/feature_summary.md
    have them (feature_extraction.py:401-502)."""
    import json as _json

    from src import feature_extraction as FE

    monkeypatch.chdir(tmp_path)
    cm = GOLD["committed_metadata"]
    e = np.random.default_rng(1).normal(size=(6, 512)).astype(np.float32)
    img = tmp_path / "mri" / "sans_label"
    img.mkdir(parents=True)
    recs = []
    for i in range(6):
        f = img / f"{i}.jpg"
        f.write_bytes(b"x")
        recs.append(FE.ImageRecord(f, Path(f"sans_label/{i}.jpg"), "unlabeled", None))
    res = FE.ExtractionResults(e, recs, [], [0.01] * 6, "random_init(seed=42)")
    FE.save_artifacts(res, FE.run_sanity_checks(e), FE.nearest_neighbor_probe(e, recs), tmp_path / "mri", "cuda")
    meta = _json.loads((tmp_path / "outputs/features/metadata.json").read_text())
    assert list(meta) == cm["keys"]
    assert list(meta["sanity_checks"]) == cm["sanity_keys"]
    assert list(meta["neighbor_probe"][0]) == cm["probe_keys"]
    assert meta["embedding_dimension"] == cm["embedding_dimension"]
    md = (tmp_path / "outputs/notes/feature_summary.md").read_text().splitlines()
    assert [ln for ln in md if ln.startswith("#")] == cm["summary_headings"]
    assert [ln.split(":")[0] for ln in md if ln.startswith("- ") and ":" in ln] == cm["summary_bullets"]
    assert np.load(tmp_path / "outputs/features/embeddings.npy").dtype == np.float32
