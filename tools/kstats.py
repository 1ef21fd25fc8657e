"""Categorised per-step kernel time from a rocprofv3 --kernel-trace --stats csv.
usage: python tools/kstats.py <run_kernel_stats.csv> <steps_in_trace> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
cat = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r['Name']; t = float(r['TotalDurationNs']) / 1e6 / steps; c = int(r['Calls']) / steps
    if n.startswith('igemm_fwd') or 'conv_fwd' in n or 'miopenSp3' in n: k = 'conv fwd (MIOpen)'
    elif n.startswith('igemm_bwd') or 'bwd_data' in n: k = 'conv dgrad (MIOpen)'
    elif n.startswith('igemm_wrw') or 'bwd_weight' in n: k = 'conv wgrad (MIOpen)'
    elif 'transpose' in n: k = 'transpose (MIOpen)'
    elif 'SubTensorOp' in n or 'OpTensor' in n: k = 'MIOpen tensor ops'
    elif 'conv1d_mfma' in n: k = 'HIP conv fwd/dgrad'
    elif 'wgrad_kernel' in n: k = 'HIP conv wgrad'
    elif 'pack16' in n: k = 'HIP pack16'
    elif 'reduce_kernel' in n: k = 'reduce'
    elif 'copy_kernel' in n or 'CatArray' in n or 'direct_copy' in n: k = 'copy/cast'
    elif 'elementwise' in n: k = 'elementwise'
    elif 'Cijk' in n: k = 'gemm (hipBLASLt)'
    else: k = 'other'
    cat[k][0] += c; cat[k][1] += t
tot = sum(v[1] for v in cat.values())
print(f"total GPU kernel time per step: {tot:.2f} ms")
for k, v in sorted(cat.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:8.2f} ms {v[0]:7.0f} calls  {k}")
print()
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:7.2f} ms {int(r['Calls'])/steps:6.0f} {r['Name'][:110]}")
