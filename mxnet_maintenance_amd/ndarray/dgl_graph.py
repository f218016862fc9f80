"""Graph operators for DGL on CSR adjacency matrices (parity: src/operator/contrib/dgl_graph.cc:761,
866, 1146, 1331, 1407, 1582): neighbourhood sampling, induced subgraphs, edge-id lookup, adjacency
and subgraph compaction.  The CSR's values are edge ids (int64).

They work directly on the compressed storage of CSRNDArray (no densification): sampling is a BFS
with per-vertex neighbour sampling on the host (the reference is CPU-only too), and ``edge_id`` is a
vectorised row search that runs wherever the CSR lives.
"""
import numpy as np
import torch

from ..base import MXNetError
from .ndarray import NDArray
from .sparse import CSRNDArray

__all__ = ['dgl_csr_neighbor_uniform_sample', 'dgl_csr_neighbor_non_uniform_sample', 'dgl_subgraph',
           'edge_id', 'dgl_adjacency', 'dgl_graph_compact']


def _parts(csr):
    if not isinstance(csr, CSRNDArray):
        raise MXNetError('expected a CSRNDArray graph')
    csr._sync()
    ptr, idx = csr._aux
    return csr._vals, idx, ptr, csr.shape


def _np1(a):
    return (a._data if isinstance(a, NDArray) else torch.as_tensor(a)).detach().cpu().numpy().reshape(-1)


def _csr(vals, indices, indptr, shape, device):
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64), device=device)     # noqa: E731
    return CSRNDArray._make(t(vals), [t(indptr), t(indices)], shape)


def _sample_neighbors(cols, eids, k, rng, prob=None):
    n = len(cols)
    if n <= k:
        return cols, eids
    if prob is None:
        pick = np.sort(rng.choice(n, size=k, replace=False))
    else:
        w = prob[cols].astype(np.float64)
        w = w / w.sum() if w.sum() > 0 else None
        pick = np.sort(rng.choice(n, size=k, replace=False, p=w))
    return cols[pick], eids[pick]


def _sample_one(vals, idx, ptr, shape, seed_ids, num_hops, num_neighbor, max_num_vertices, prob, rng):
    ptr = ptr.cpu().numpy()
    idx = idx.cpu().numpy()
    vals = vals.cpu().numpy()
    seen = set()
    queue = []                      # (vertex, layer), BFS order; also the sampled vertex set
    for s in seed_ids:
        s = int(s)
        if s not in seen:
            seen.add(s)
            queue.append((s, 0))
    neigh = {}
    i = 0
    while i < len(queue) and len(seen) < max_num_vertices:
        v, layer = queue[i]
        i += 1
        if layer >= num_hops:
            continue
        cols, eids = _sample_neighbors(idx[ptr[v]:ptr[v + 1]], vals[ptr[v]:ptr[v + 1]], num_neighbor, rng, prob)
        neigh[v] = (cols, eids)
        for c in cols:
            if len(seen) >= max_num_vertices:
                break
            c = int(c)
            if c not in seen:
                seen.add(c)
                queue.append((c, layer + 1))
    queue.sort(key=lambda p: p[0])
    n = len(queue)
    sample_id = np.full(max_num_vertices + 1, -1, dtype=np.int64)
    layer = np.full(max_num_vertices, -1, dtype=np.int64)
    for j, (v, l) in enumerate(queue):
        sample_id[j] = v
        layer[j] = l
    sample_id[max_num_vertices] = n
    indptr = [0]
    cols_out, eids_out = [], []
    for v, _ in queue:
        c, e = neigh.get(v, ((), ()))
        cols_out.extend(int(x) for x in c)
        eids_out.extend(int(x) for x in e)
        indptr.append(len(cols_out))
    indptr.extend([len(cols_out)] * (max_num_vertices - n))
    return sample_id, (eids_out, cols_out, indptr), layer


def _sampler(csr, seeds, num_hops, num_neighbor, max_num_vertices, prob=None):
    vals, idx, ptr, shape = _parts(csr)
    rng = np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))
    p = _np1(prob).astype(np.float64) if prob is not None else None
    ids, csrs, probs, layers = [], [], [], []
    for s in seeds:
        sid, (e, c, ip), layer = _sample_one(vals, idx, ptr, shape, _np1(s), num_hops, num_neighbor,
                                             max_num_vertices, p, rng)
        dev = vals.device
        ids.append(NDArray(torch.as_tensor(sid, device=dev)))
        csrs.append(_csr(e, c, ip, (max_num_vertices, shape[1]), dev))
        layers.append(NDArray(torch.as_tensor(layer, device=dev)))
        if p is not None:
            sp = np.zeros(max_num_vertices, dtype=np.float32)
            n = int(sid[-1])
            sp[:n] = p[sid[:n]]
            probs.append(NDArray(torch.as_tensor(sp, device=dev)))
    return ids + csrs + (probs if p is not None else []) + layers


def dgl_csr_neighbor_uniform_sample(csr, *seeds, num_args=None, num_hops=1, num_neighbor=2,
                                    max_num_vertices=100):
    """Per seed array: BFS up to ``num_hops`` sampling at most ``num_neighbor`` neighbours per vertex
    uniformly; returns [sample_id...] + [sub_csr...] + [layer...] (sample_id[-1] = #vertices)."""
    return _sampler(csr, seeds, num_hops, num_neighbor, max_num_vertices)


def dgl_csr_neighbor_non_uniform_sample(csr, probability, *seeds, num_args=None, num_hops=1, num_neighbor=2,
                                        max_num_vertices=100):
    """As the uniform sampler with neighbours drawn in proportion to ``probability`` (per vertex);
    also returns the sampled vertices' probabilities."""
    return _sampler(csr, seeds, num_hops, num_neighbor, max_num_vertices, prob=probability)


def dgl_subgraph(graph, *vertex_sets, return_mapping=False, num_args=None):
    """Induced subgraph(s) on sorted vertex id arrays: CSR with new edge ids 0..nnz-1, and with
    ``return_mapping`` a second CSR holding the original edge ids."""
    vals, idx, ptr, shape = _parts(graph)
    ptr_n, idx_n, vals_n = ptr.cpu().numpy(), idx.cpu().numpy(), vals.cpu().numpy()
    subs, maps = [], []
    for vs in vertex_sets:
        v = _np1(vs).astype(np.int64)
        if np.any(v[1:] < v[:-1]):
            raise MXNetError('The input vertex list has to be sorted')
        if len(v) and int(v.max()) >= shape[0]:
            raise MXNetError('Vertex Id %d isn\'t in a graph of %d vertices' % (int(v.max()), shape[0]))
        new_id = {int(x): i for i, x in enumerate(v)}
        indptr, cols, old = [0], [], []
        for x in v:
            for j in range(ptr_n[x], ptr_n[x + 1]):
                c = int(idx_n[j])
                if c in new_id:
                    cols.append(new_id[c])
                    old.append(int(vals_n[j]))
            indptr.append(len(cols))
        n = len(v)
        subs.append(_csr(np.arange(len(cols)), cols, indptr, (n, n), vals.device))
        maps.append(_csr(old, cols, indptr, (n, n), vals.device))
    out = subs + (maps if return_mapping else [])
    return out[0] if len(out) == 1 else out


def edge_id(data, u, v):
    """out[i] = data[u[i], v[i]] when that edge exists, else -1 (vectorised search in CSR rows)."""
    vals, idx, ptr, shape = _parts(data)
    uu = (u._data if isinstance(u, NDArray) else torch.as_tensor(u)).to(idx.device).long().reshape(-1)
    vv = (v._data if isinstance(v, NDArray) else torch.as_tensor(v)).to(idx.device).long().reshape(-1)
    out = torch.full(uu.shape, -1.0, dtype=vals.dtype if vals.is_floating_point() else torch.float32,
                     device=idx.device)
    if idx.numel():
        start, end = ptr[uu], ptr[uu + 1]
        width = int((ptr[1:] - ptr[:-1]).max())
        offs = torch.arange(width, device=idx.device)
        pos = start.unsqueeze(1) + offs.unsqueeze(0)
        valid = pos < end.unsqueeze(1)
        posc = torch.where(valid, pos, torch.zeros_like(pos))
        hit = valid & (idx[posc] == vv.unsqueeze(1))
        found = hit.any(1)
        first = torch.argmax(hit.to(torch.int8), dim=1)
        got = vals[posc.gather(1, first.unsqueeze(1)).squeeze(1)].to(out.dtype)
        out = torch.where(found, got, out)
    return NDArray(out)


def dgl_adjacency(data):
    """The adjacency matrix of an edge-id CSR: same structure, every stored value 1.0 (float32)."""
    vals, idx, ptr, shape = _parts(data)
    return CSRNDArray._make(torch.ones(vals.shape, dtype=torch.float32, device=vals.device),
                            [ptr.clone(), idx.clone()], shape)


def dgl_graph_compact(*args, graph_sizes=(), return_mapping=False, num_args=None):
    """Compact sampled subgraph CSRs (rows = sampled vertices, columns = parent ids) into
    graph_size x graph_size CSRs whose columns index the sampled vertex list."""
    k = len(args) // 2
    graphs, vids = args[:k], args[k:]
    if isinstance(graph_sizes, (int, np.integer)):
        graph_sizes = (graph_sizes,)
    graph_sizes = [int(np.asarray(g).reshape(-1)[0]) if not isinstance(g, (int, np.integer)) else int(g)
                   for g in graph_sizes]
    outs, maps = [], []
    for g, vid, n in zip(graphs, vids, graph_sizes):
        vals, idx, ptr, _shape = _parts(g)
        ids = _np1(vid)
        if int(ids[-1]) != n:
            raise MXNetError('dgl_graph_compact: graph size %d does not match the sample count %d'
                             % (n, int(ids[-1])))
        id_map = {int(x): i for i, x in enumerate(ids[:n])}
        cols = [id_map[int(c)] for c in idx.cpu().numpy()]
        indptr = ptr.cpu().numpy()[:n + 1]
        outs.append(_csr(np.arange(len(cols)), cols, indptr, (n, n), vals.device))
        maps.append(_csr(vals.cpu().numpy(), cols, indptr, (n, n), vals.device))
    res = outs + (maps if return_mapping else [])
    return res[0] if len(res) == 1 else res
