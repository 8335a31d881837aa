"""GPU discovery and placement without importing torch or initialising HIP.

The coordinator (the notebook kernel) must not need torch — it may run on an interpreter that
has IPython but no PyTorch — and must never create a HIP context of its own (that would pin
memory on GPU 0 and, on this pool, initialising the GPU in a process that later execs is
forbidden).  So devices are enumerated from the KFD topology in sysfs, which is also where the
xGMI link table comes from.

Reference: GPU ids are validated with ``torch.cuda.device_count()`` in the kernel
(``magic.py:455-488``) and each worker calls ``set_device(gpu_id)`` while exporting
``LOCAL_RANK=rank`` (``worker.py:129, 138``) — the mismatch behind bug D-12.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional

KFD_NODES = Path("/sys/class/kfd/kfd/topology/nodes")
IOLINK_TYPE_XGMI = 11
IOLINK_TYPE_PCIE = 2


def _read_props(path: Path) -> Dict[str, int]:
    out: Dict[str, int] = {}
    try:
        for line in path.read_text().splitlines():
            parts = line.split()
            if len(parts) == 2:
                try:
                    out[parts[0]] = int(parts[1])
                except ValueError:
                    pass
    except OSError:
        pass
    return out


@dataclass
class KfdGpu:
    node: int
    gfx_target_version: int
    simd_count: int
    drm_render_minor: int
    unique_id: int
    location_id: int
    links: List[Dict[str, int]] = field(default_factory=list)

    @property
    def gfx_arch(self) -> str:
        v = self.gfx_target_version
        major, minor, step = v // 10000, (v // 100) % 100, v % 100
        return f"gfx{major}{minor:x}{step:x}" if v else "unknown"


def kfd_gpus() -> List[KfdGpu]:
    """All GPU nodes in KFD topology order (the order ROCr enumerates them)."""
    gpus: List[KfdGpu] = []
    if not KFD_NODES.exists():
        return gpus
    nodes = sorted((p for p in KFD_NODES.iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
    for n in nodes:
        props = _read_props(n / "properties")
        if props.get("simd_count", 0) <= 0:
            continue  # CPU node
        g = KfdGpu(node=int(n.name), gfx_target_version=props.get("gfx_target_version", 0),
                   simd_count=props.get("simd_count", 0), drm_render_minor=props.get("drm_render_minor", -1),
                   unique_id=props.get("unique_id", 0), location_id=props.get("location_id", 0))
        links_dir = n / "io_links"
        if links_dir.exists():
            for l in sorted(links_dir.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else 0):
                g.links.append(_read_props(l / "properties"))
        gpus.append(g)
    return gpus


def _parse_list(v: Optional[str]) -> Optional[List[str]]:
    if v is None:
        return None
    v = v.strip()
    if v == "":
        return []
    return [x.strip() for x in v.split(",") if x.strip()]


def parent_visible() -> Optional[List[str]]:
    """The device filter this process already runs under (HIP_VISIBLE_DEVICES wins over
    CUDA_VISIBLE_DEVICES in the HIP runtime).  ROCR_VISIBLE_DEVICES is applied below both and
    is passed through to workers untouched."""
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = _parse_list(os.environ.get(k))
        if v is not None:
            return v
    return None


def visible_gpu_count() -> int:
    n = len(kfd_gpus())
    rocr = _parse_list(os.environ.get("ROCR_VISIBLE_DEVICES"))
    if rocr is not None:
        n = min(n, len(rocr))
    pv = parent_visible()
    if pv is not None:
        n = min(n, len(pv))
    return n


def worker_visible_devices(gpu_ids: List[int]) -> str:
    """HIP_VISIBLE_DEVICES value for the workers: the distinct assigned GPUs in rank order,
    translated through the parent's own filter so ids mean what they mean in the kernel."""
    uniq: List[int] = []
    for g in gpu_ids:
        if g not in uniq:
            uniq.append(g)
    pv = parent_visible()
    if pv is not None:
        return ",".join(pv[g] for g in uniq)
    return ",".join(str(g) for g in uniq)


def local_device_index(gpu_ids: List[int], rank: int) -> int:
    uniq: List[int] = []
    for g in gpu_ids:
        if g not in uniq:
            uniq.append(g)
    return uniq.index(gpu_ids[rank])


def xgmi_matrix(gpus: Optional[List[KfdGpu]] = None) -> Dict[str, object]:
    """Link table between GPU nodes: type (xgmi/pcie), hops, weight and bandwidth (MB/s)."""
    gpus = gpus if gpus is not None else kfd_gpus()
    node_to_idx = {g.node: i for i, g in enumerate(gpus)}
    rows = []
    for i, g in enumerate(gpus):
        for l in g.links:
            dst = l.get("node_to")
            if dst not in node_to_idx:
                continue
            t = l.get("type", 0)
            rows.append({"src": i, "dst": node_to_idx[dst],
                         "type": "xgmi" if t == IOLINK_TYPE_XGMI else ("pcie" if t == IOLINK_TYPE_PCIE else str(t)),
                         "hops": l.get("num_hops", 0), "weight": l.get("weight", 0),
                         "min_bw_mbs": l.get("min_bandwidth", 0), "max_bw_mbs": l.get("max_bandwidth", 0)})
    return {"n_gpus": len(gpus), "links": rows}
