"""Summarise a rocprofv3 kernel trace: per-step kernel time by family."""
import csv, sys, collections
path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
fam = collections.defaultdict(lambda: [0.0, 0])
def family(n):
    for k in ('conv_gemm_kernelILi', 'conv_glds_kernelILi', 'conv_glds_kernel<'):
        if k in n:
            mode = n.split(k)[1][0]
            return {'0': 'conv_fwd', '1': 'conv_dgrad', '2': 'conv_wgrad'}[mode]
    for k in ['wgrad_reduce', 'bn_apply', 'bn_bwd_apply', 'bn_bwd_reduce', 'bn_bwd_finalize', 'bn_finalize',
              'maxpool_fwd', 'maxpool_bwd', 'augment', 'resize_h', 'weight_prep', 'adamw', 'avgpool_fc_fwd',
              'avgpool_fc_bwd', 'fc_bwd_weight', 'semi_loss', 'cross_entropy', 'nchw_to_nhwc']:
        if k in n:
            return k
    return 'other:' + n[:50]
tot = 0
for r in rows:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    f = fam[family(r['Kernel_Name'])]
    f[0] += d; f[1] += 1; tot += d
for k, (t, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f"{t/steps/1e3:8.3f} ms/step {100*t/tot:5.1f}%  n/step={n/steps:6.1f}  {k}")
print(f"total {tot/steps/1e3:.3f} ms/step")
