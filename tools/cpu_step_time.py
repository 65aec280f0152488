"""Host-side cost of one eager SemiStep (GPU box): time to draw the
augmentation parameters and to enqueue a whole step (no synchronisation),
against the GPU time per step."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402
from ssip import SSIPResNet, replace_fc  # noqa: E402
from ssip.semi_step import SemiStep  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(42)
model = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
step = SemiStep(model, lr=1e-4, weight_decay=1e-4, tau=0.7, image_size=224, graph=False)
g = torch.Generator(device="cpu").manual_seed(1000)
x_l = torch.randint(0, 256, (128, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
x_u = torch.randint(0, 256, (128, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
y_l = torch.randint(0, 2, (128,), generator=g).to(dev)
for _ in range(5):
    step(x_l, y_l, x_u)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    p = step.draw_params(128, 128)
t1 = time.perf_counter()
print(f"draw_params: {(t1 - t0) / 20 * 1e3:.2f} ms", flush=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    step(x_l, y_l, x_u)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"enqueue 10 steps: {(t1 - t0) / 10 * 1e3:.2f} ms/step host, {(t2 - t0) / 10 * 1e3:.2f} ms/step wall", flush=True)

if os.environ.get("SSIP_CPROFILE"):
    import cProfile, pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        step(x_l, y_l, x_u)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
