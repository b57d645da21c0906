"""Process meshes (capability parity with init_device_mesh / DeviceMesh of the reference,
scripts/03_tensor_parallel_tp/01_device_mesh_basics.py:29-73, fsdp_tp/fsdp_tp_example.py:120-131).

``Mesh((dp, tp), ("dp", "tp"))`` lays ranks out row-major with the LAST dim fastest-varying, so a tp group is a
block of consecutive ranks.  On one 8-GPU MI355X node every pair of GPUs is one xGMI hop, so unlike the
reference's NVLink-island rule ("keep TP inside a node") any grouping is topologically equivalent; consecutive
blocks are kept so multi-node extensions keep TP intra-node.

Sub-groups are created eagerly for every dim (all ranks call ``new_group`` in the same order, as c10d
requires).  ``torch_mesh()`` returns the equivalent torch DeviceMesh for users of DTensor APIs.
"""
from __future__ import annotations

import itertools
from typing import Sequence

import torch
import torch.distributed as dist


class Mesh:
    def __init__(self, shape: Sequence[int], names: Sequence[str], backend: str | None = None):
        assert len(shape) == len(names)
        self.shape = tuple(int(s) for s in shape)
        self.names = tuple(names)
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        n = 1
        for s in self.shape:
            n *= s
        assert n == world, f"mesh {self.shape} needs {n} ranks, world is {world}"
        self.rank = rank
        self.coords = self._coords(rank)
        self.groups: dict[str, object] = {}
        self.group_ranks: dict[str, list[int]] = {}
        for d, name in enumerate(self.names):
            others = [range(s) for i, s in enumerate(self.shape) if i != d]
            for combo in itertools.product(*others):
                ranks = []
                for k in range(self.shape[d]):
                    c = list(combo)
                    c.insert(d, k)
                    ranks.append(self._rank_of(c))
                g = dist.new_group(ranks, backend=backend) if dist.is_initialized() and world > 1 else None
                if rank in ranks:
                    self.groups[name] = g
                    self.group_ranks[name] = ranks

    def _coords(self, r):
        c = []
        for s in reversed(self.shape):
            c.append(r % s)
            r //= s
        return tuple(reversed(c))

    def _rank_of(self, coords):
        r = 0
        for c, s in zip(coords, self.shape):
            r = r * s + c
        return r

    def size(self, name: str) -> int:
        return self.shape[self.names.index(name)]

    def local_rank(self, name: str) -> int:
        return self.coords[self.names.index(name)]

    def group(self, name: str):
        return self.groups[name]

    def __getitem__(self, name):
        return self.groups[name]

    def torch_mesh(self, device_type: str = "cuda"):
        from torch.distributed.device_mesh import init_device_mesh

        return init_device_mesh(device_type, self.shape, mesh_dim_names=self.names)

    def __repr__(self):
        return f"Mesh(shape={self.shape}, names={self.names}, rank={self.rank}, coords={self.coords})"


class DeviceMesh2D(Mesh):
    """(dp, tp) mesh with tp fastest-varying: ``dp_group``/``tp_group``/``dp_rank``/``tp_rank``."""

    def __init__(self, dp: int, tp: int, backend: str | None = None):
        super().__init__((dp, tp), ("dp", "tp"), backend)
        self.dp_group, self.tp_group = self.groups["dp"], self.groups["tp"]
        self.dp_rank, self.tp_rank = self.coords
        self.dp, self.tp = dp, tp


def mesh_sanity_check(mesh: Mesh, device=None) -> dict:
    """all-reduce of the rank ids over each mesh dim; returns {dim: (got, expected)} (01_device_mesh_basics.py:82-87)."""
    out = {}
    dev = device or torch.device("cpu")
    for name in mesh.names:
        t = torch.tensor([float(mesh.rank)], device=dev)
        if mesh.groups.get(name) is not None:
            dist.all_reduce(t, group=mesh.groups[name])
        out[name] = (t.item(), float(sum(mesh.group_ranks[name])))
    return out
