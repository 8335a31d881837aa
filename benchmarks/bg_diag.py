import contextlib, sys, traceback, warnings, torch
warnings.simplefilter('always')
sys.path.insert(0, "/root/repo")
sys.path.insert(0, ".")
from nbdistributed_amd import ops
import tests.test_gpu_block_graphs as T
dev = torch.device("cuda")
base = T._model(dev, layers=2, seed=7)
batches = T._batches(dev, n=1)
from nbdistributed_amd.graphs import GraphedStep
import nbdistributed_amd.graphs as GR
if '--suspend' not in sys.argv:
    GR._suspend_block_graphs = contextlib.nullcontext  # the autograd-history fix alone
import copy
for graphs in (False, True):
    ops.block_graphs(graphs)
    m = copy.deepcopy(base)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True, foreach=False)
    def step(x, y):
        loss = m(x, torch.ones_like(x), y)[0]
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        return loss.detach()
    try:
        call = GraphedStep(step, batches[0], warmup=3, optimizers=[opt])
        ls = torch.stack([call(*batches[0]).clone() for _ in range(5)])
        torch.cuda.synchronize()
        print(graphs, ls.tolist(), ops.block_graphs_stats(), flush=True)
    except Exception:
        traceback.print_exc()
        print("stats", ops.block_graphs_stats(), flush=True)
        sys.exit(1)
