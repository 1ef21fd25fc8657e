"""Graph capture of the train step with the flat RCCL gradient all-reduce
(TrainStep(allreduce=True)).  Run under torchrun on the GPU box, e.g.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29531 tools/rccl_capture_check.py
(one rank still launches the RCCL all-reduce kernels inside the graph)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

rank = int(os.environ["RANK"]); local = int(os.environ["LOCAL_RANK"])
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
dist.init_process_group("nccl")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, capturable=True, allreduce=True)
assert st.allreduce
batch = [t.to(dev) for t in synthetic_batch(hps, int(os.environ.get("B", "16")), seed=rank)]
t0 = time.perf_counter()
st.capture(batch, warmup=2)
torch.cuda.synchronize()
print(f"rank {rank}: captured in {time.perf_counter() - t0:.1f}s", flush=True)
for i in range(5):
    out = st.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(5):
    out = st.replay()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 5
print(f"rank {rank}: replay {dt*1e3:.1f} ms loss_g={float(out['loss_gen_all']):.3f} "
      f"loss_d={float(out['loss_disc']):.3f}", flush=True)
assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_disc"])
dist.destroy_process_group()
print("RCCL_CAPTURE_OK", flush=True)
