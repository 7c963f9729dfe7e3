"""The reference's material-prediction GCN (ipt.py:26-83) on PyTorch-ROCm
without DGL (DGL is not installed and has no ROCm build here).

DGL supplied three things, restated with plain tensor ops:
* ``dgl.graph((src, dst))`` + ``dgl.add_self_loop`` -> :class:`Graph` (edge
  lists, edge weights, node features) built by :func:`build_graph`;
* ``update_all(src_mul_edge('node_feats', 'edge_feats'), sum)`` -> one
  ``index_add_`` over the edge list (:meth:`Graph.propagate`): reduced[dst]
  = sum over edges (src -> dst) of h[src] * w;
* ``dgl.batch`` -> :func:`batch` (node indices offset per graph).

``dgl.add_self_loop`` fills the new edges' feature with 0 in the DGL releases
of the reference's time (0.5-0.8) and with 1 from 0.9 on; the reference pins
no version, so the fill value is a parameter (default 0: the self loop then
contributes nothing to the sum).  Parity with DGL itself is unpinned; the
tests pin the message passing against a dense numpy restatement.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

P_MIN = 1e-3  # ipt.py:24


@dataclass
class Graph:
    src: torch.Tensor         # int64 [E]
    dst: torch.Tensor         # int64 [E]
    edge_w: torch.Tensor      # float32 [E]
    node_feats: torch.Tensor  # float32 [nodes, 3]

    @property
    def num_nodes(self) -> int:
        return int(self.node_feats.shape[0])

    def to(self, device) -> "Graph":
        return Graph(self.src.to(device), self.dst.to(device), self.edge_w.to(device), self.node_feats.to(device))

    def propagate(self, h: torch.Tensor) -> torch.Tensor:
        """update_all(fn.src_mul_edge('node_feats','edge_feats','msg'), fn.sum('msg','reduced'))
        (ipt.py:60-63): reduced[v] = sum over edges u -> v of h[u] * w(u, v)."""
        msg = h.index_select(0, self.src) * self.edge_w.unsqueeze(-1)
        return torch.zeros_like(h).index_add_(0, self.dst, msg)


def build_graph(w, pixel, light=None, p_min: float = P_MIN, self_loop_fill: float = 0.0) -> Graph:
    """ipt.py:68-83.  w: (nT+1, nT) transport weights (row = destination
    triangle, last row = the eye), pixel: (nT+1, nT, 3); light is unused, as in
    the reference.  Nodes are triangles, node features the eye row's pixel
    colours, edges src -> dst for every kept weight w[dst, src] (row-normalised,
    entries below p_min dropped), plus one self loop per node."""
    w = np.array(w, dtype=np.float64, copy=True)  # the reference mutates its input; we do not
    pixel = np.asarray(pixel, dtype=np.float64)
    w[w < p_min] = 0.0
    w_sum = w.sum(axis=-1, keepdims=True)
    w = w / np.where(w_sum != 0, w_sum, np.ones_like(w_sum))
    w, w_eye = w[:-1], w[-1]
    pixel_eye = pixel[-1]
    dst, src = w.nonzero()  # row-major, the order of w[w != 0]
    n = len(w_eye)
    loops = np.arange(n)
    src = np.concatenate([src, loops])
    dst = np.concatenate([dst, loops])
    ew = np.concatenate([w[w != 0], np.full(n, self_loop_fill)])
    return Graph(torch.from_numpy(src.astype(np.int64)), torch.from_numpy(dst.astype(np.int64)),
                 torch.from_numpy(ew.astype(np.float32)), torch.from_numpy(pixel_eye.astype(np.float32)))


def batch(graphs: Sequence[Graph]) -> Graph:
    """dgl.batch: one disjoint graph, node ids of graph k offset by the nodes before it."""
    off, src, dst = 0, [], []
    for g in graphs:
        src.append(g.src + off)
        dst.append(g.dst + off)
        off += g.num_nodes
    return Graph(torch.cat(src), torch.cat(dst), torch.cat([g.edge_w for g in graphs]),
                 torch.cat([g.node_feats for g in graphs]))


class MPL(nn.Module):
    """ipt.py:50-66: h <- act(Linear(cat(h, sum of weighted neighbour h)))."""

    def __init__(self, in_feats: int, out_feats: int, activation=None):
        super().__init__()
        self.linear = nn.Linear(in_feats * 2, out_feats)
        self.activation = activation

    def forward(self, g: Graph, h: torch.Tensor) -> torch.Tensor:
        h = self.linear(torch.cat((h, g.propagate(h)), dim=-1))
        return self.activation(h) if self.activation is not None else h


class GCN(nn.Module):
    """ipt.py:26-48: lift (tanh) -> 3 x MPL(relu) -> out (sigmoid); L1 loss."""

    def __init__(self, in_feats: int = 3, out_feats: int = 3, hidden: int = 100):
        super().__init__()
        self.lift = nn.Linear(in_feats, hidden)
        self.network = nn.ModuleList([MPL(hidden, hidden, F.relu) for _ in range(3)])
        self.out = nn.Linear(hidden, out_feats)

    def forward(self, g: Graph) -> torch.Tensor:
        h = self.lift(g.node_feats).tanh()
        for layer in self.network:
            h = layer(g, h)
        return self.out(h).sigmoid()

    @staticmethod
    def loss(preds: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        return (preds - labels).abs().mean()


def train(graphs: List[Graph], labels: List[torch.Tensor], epochs: int, lr: float = 1e-4, device=None,
          log_every: int = 0, seed: int = 0) -> GCN:
    """ipt.py:106-124: Adam on the batched training graphs, one step per epoch."""
    torch.manual_seed(seed)
    device = torch.device(device) if device is not None else torch.device("cpu")
    model = GCN(3, 3).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    x = batch(graphs).to(device)
    y = torch.cat([torch.as_tensor(l, dtype=torch.float32) for l in labels], dim=0).to(device)
    for i in range(epochs):
        loss = model.loss(model(x), y)
        if log_every and (i + 1) % log_every == 0:
            print((i + 1) // log_every, float(loss.detach().cpu()), flush=True)
        opt.zero_grad()
        loss.backward()
        opt.step()
    return model
