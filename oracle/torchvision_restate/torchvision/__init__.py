"""ORACLE (test infrastructure only): restatement of the parts of
torchvision (>=0.15, absent from this image) that the reference calls:
models.resnet18/resnet50 (+ weights enum), transforms.{Compose, Resize,
CenterCrop, RandomHorizontalFlip, RandomRotation, ToTensor, Normalize} on
PIL images, datasets.ImageFolder.  Used (a) as the CPU reference model and
(b) put on sys.path as `torchvision` so the reference's own modules import
for golden-vector generation (tests/golden/make_goldens.py)."""
from . import datasets, models, transforms  # noqa: F401

__version__ = "0.0-ssip-oracle-restatement"
