import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ.setdefault("RANK","0"); os.environ.setdefault("WORLD_SIZE","1"); os.environ.setdefault("MASTER_ADDR","127.0.0.1"); os.environ.setdefault("MASTER_PORT","29555")
from nbdistributed_amd.parallel.backend import init_data_plane
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
init_data_plane("rccl", 0, 1, dev)
m = GPT2(GPT2Config.small()).to(dev).to(torch.bfloat16)
w = NbdDDP(m, flat_params=True, grad_mode="bucket"); opt = FlatAdamW(w, lr=3e-4)
x = torch.randint(0, 50257, (8, 1024), device=dev)
def step():
    _, loss = w(x, x, return_logits=False); loss.backward(); opt.step(); opt.zero_grad(set_to_none=True)
for _ in range(3): step()
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=False) as p:
    step(); torch.cuda.synchronize()
print(p.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=45, max_name_column_width=60))
