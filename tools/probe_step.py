"""Quick throughput probe of the ResNet-18 train step (dev tool)."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "semi-supervised-image-processing_amd"))
import torch
from ssip import SSIPResNet, replace_fc, ops
from ssip.optim import AdamW

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
torch.manual_seed(42)
m = replace_fc(SSIPResNet("resnet18", 1000, dtype=dtype), 2).cuda().train()
arena = m.flatten_parameters()
opt = AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4, arena=arena)
x = torch.randn(B, 3, 224, 224, device="cuda")
y = torch.randint(0, 2, (B,), device="cuda")
def step():
    opt.zero_grad(set_to_none=True)
    out = m(x)
    loss, dl, pred = ops.cross_entropy(out.detach(), y)
    out.backward(dl)
    opt.step()
for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"B={B} dtype={dtype} step_ms={dt*1e3:.2f} img/s={B/dt:.1f}")
