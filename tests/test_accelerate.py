"""The reference notebook's workflow: HF accelerate inside %%distributed cells (CPU/gloo here;
the GPU variant with backend "rccl" is in test_gpu_session.py)."""
import pytest

from nbdistributed_amd.session import Session

ACCEL = """
from accelerate import Accelerator
from accelerate.utils import set_seed
import torch.nn as nn
from torch.utils.data import TensorDataset, DataLoader
from nbdistributed_amd.models import synthetic_mrpc
set_seed(42)
acc = Accelerator(cpu=(device.type == 'cpu'))
ids, mask, labels = synthetic_mrpc(n=64, seq_len=16, vocab=100)
dl = DataLoader(TensorDataset(ids, labels), batch_size=8, shuffle=True)
model = nn.Sequential(nn.Embedding(100, 16), nn.Flatten(), nn.Linear(16 * 16, 2))
opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
model, opt, dl = acc.prepare(model, opt, dl)
for x, y in dl:
    loss = nn.functional.cross_entropy(model(x), y)
    acc.backward(loss)
    opt.step(); opt.zero_grad()
preds = acc.gather_for_metrics(model(x).argmax(-1))
(acc.num_processes, acc.process_index, int(preds.numel()), str(acc.device))
"""


def test_accelerate_prepare_backward_gather_on_gloo():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    try:
        r = s.execute(ACCEL, render=False)
        assert r.results[0]["echo"].startswith("(2, 0, 16,")
        assert r.results[1]["echo"].startswith("(2, 1, 16,")
    finally:
        s.shutdown()
