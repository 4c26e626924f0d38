"""The headline workload (BASELINE.json metric), built per rank.

The GAT layer-1 aggregate block [3, 11, 12] -- scatter C -> applyedge MUL -> gather ADD, lowered
by interpret() to one COMP_MUL_COMP_ADD with the scatter's FETCH removed (code/interpreter.py:
575-636, 764-802; Inst_fused `FinalVersion For Paper/hardware_info.yaml:35-38`):
    Y[i, :] = sum_{e -> i} alpha[e, head(c)] * X1[src(e), :]
on a Reddit-shaped CSR (N = 232,965, E = 114,615,892), F = 128 fp32 = 8 heads x 16,
alpha = per-head softmax over each destination's in-edges (GAT ops 6-10) of N(0, 1) logits.

Every input is a pure function of (seed, id) (graph.CounterCSR, graph.hash_normal): a rank of the
multi-GPU bench generates only its row group's edges and its column slice of X, and any rank can
regenerate any X row or edge bit for bit (the parity check).  On one GPU the shard is the whole
graph.
"""
import torch

from . import distributed, graph as G, partition

N_REDDIT, E_REDDIT = 232965, 114615892
F, HEADS = 128, 8
SEED = 0
STREAM_X, STREAM_LOGIT = 2, 3


def alg_bytes(n_rows, nnz, f=F, heads=HEADS):
    """per edge 4 (col idx) + 4*H (alpha) + 4*F (gathered X row); per node 8 (indptr) + 4*F (Y)."""
    return nnz * (4 + 4 * heads + 4 * f) + n_rows * (8 + 4 * f)


def compulsory_bytes(n_rows, n_cols, nnz, f=F, heads=HEADS):
    """Bytes that must cross HBM once: col idx + alpha per edge, indptr + Y per row, X once."""
    return nnz * (4 + 4 * heads) + n_rows * (8 + 4 * f) + n_cols * 4 * f


def x_rows(ids, device, seed=SEED, f=F):
    """X1[ids, :] ~ N(0, 1), fp32 (any subset of the [N, F] table)."""
    ids = torch.as_tensor(ids, device=device, dtype=torch.int64)
    k = ids[:, None] * f + torch.arange(f, device=device, dtype=torch.int64)
    return G.hash_normal(k, seed, STREAM_X)


def alpha_rows(lip, gen, device, seed=SEED, heads=HEADS):
    """alpha [E_rows, H] fp32 of a row range in CSR order: softmax over each row's in-edges, per head,
    of N(0, 1) logits keyed by the edge's generation id.  Row sums in fp64, one segment per row summed
    in edge order (deterministic, and the same whatever row range a rank generates), one fp32 divide
    per edge.  (Until round 5 the sums were differences of one fp64 prefix sum over the rank's
    edges, whose rounding depended on where the rank's range started.)

    On the device this is one libgta launch (gta_synth_alpha: a wave per row, no device-wide scan;
    round 6, after torch's segment_reduce / repeat_interleave stalled the 8-process one-GPU
    rehearsal); alpha_rows_torch is the same formula in torch ops, the CPU path and the GPU test's
    bitwise reference (tests/test_gpu_metric.py)."""
    if gen.numel() == 0:
        return torch.empty(0, heads, device=device)
    if torch.device(device).type == "cuda":
        from . import ops
        return ops.synth_alpha(lip.to(device), gen.to(device), heads, seed, STREAM_LOGIT)
    return alpha_rows_torch(lip, gen, device, seed, heads)


def alpha_rows_torch(lip, gen, device, seed=SEED, heads=HEADS):
    """alpha_rows in torch ops (exp of the hashed logits, torch.segment_reduce's fp64 row sums)."""
    if gen.numel() == 0:
        return torch.empty(0, heads, device=device)
    k = gen[:, None] * heads + torch.arange(heads, device=device, dtype=torch.int64)
    ex = torch.exp(G.hash_normal(k, seed, STREAM_LOGIT))
    del k
    s = torch.segment_reduce(ex.double(), "sum", lengths=lip[1:] - lip[:-1], axis=0).to(torch.float32)  # [n_rows, H]
    row = torch.repeat_interleave(torch.arange(lip.numel() - 1, device=device), lip[1:] - lip[:-1])
    return ex.div_(s[row])


def column_counts(n, e, device, seed=SEED, step=1 << 24):
    """The whole graph's per-column nnz (the column sums of the tile metadata, code/preprocessing.py:
    12-40) without a process group: every edge's source is a pure function of its id, so one
    process can count them all, `step` edges at a time.  Equal to what Shard's count_reduce
    all-reduces from every rank's rows."""
    csr = G.CounterCSR(n, e, seed)
    counts = torch.zeros(n, dtype=torch.int64, device=device)
    for e0 in range(0, e, step):
        counts += torch.bincount(csr.sources(e0, min(e, e0 + step), device), minlength=n)
    return counts


class Shard:
    """Rank `rank`'s part of the metric workload on a pr x pc grid (distributed.GridShard layout):
    graph (its tile as a CSR over its row group's padded rows, local source ids), x (X1 rows of its
    column group), alpha (its tile's edges).  `count_reduce(counts)` sums the per-column nnz
    histogram over the ranks (an all-reduce; None on one rank): the column cuts come from the
    whole graph's tile metadata (column sums of calculate_sparsity, code/preprocessing.py:12-40)
    although each rank generated only its rows.  `col_counts`: that whole-graph histogram given
    directly (column_counts: a rank's tile rebuilt alone, e.g. by bench's PMC child)."""

    def __init__(self, n, e, rank, pr, pc, chunks, device, seed=SEED, count_reduce=None, keep_rows=True,
                 note=None, fracs=None, col_counts=None):
        note = note or (lambda msg: None)
        self.n, self.e, self.seed, self.device = n, e, seed, device
        self.csr = G.CounterCSR(n, e, seed)
        self.rcuts = distributed.row_cuts_ip(torch.from_numpy(self.csr.indptr_np), pr)
        i = rank // pc
        r0, r1 = self.rcuts[i], self.rcuts[i + 1]
        self.e0 = int(self.csr.indptr_np[r0])
        lip, src, gen = self.csr.rows(r0, r1, device)
        note(f"row group {i}: rows [{r0}, {r1}), {src.numel()} edges generated")
        alpha = alpha_rows(lip, gen, device, seed)
        del gen
        note(f"row group {i}: alpha [{alpha.shape[0]}, {alpha.shape[1]}] ready")
        if pc > 1 and col_counts is not None:
            ccuts = [int(c) for c in partition.cuts_from_counts(col_counts.to(device), pc)]
        elif pc > 1:
            counts = torch.bincount(src, minlength=n)
            if count_reduce is not None:
                counts = count_reduce(counts) // pc  # every rank of a row group added the same counts
                note("column counts summed over the ranks")
            ccuts = [int(c) for c in partition.cuts_from_counts(counts, pc)]
            del counts
        else:
            ccuts = [0, n]
        self.grid = distributed.GridShard.from_rows(self.rcuts, ccuts, rank, pr, pc, lip, src, chunks, self.e0,
                                                    fracs=fracs)
        g = self.grid
        self.graph = g.graph
        self.alpha = alpha[g.local_edge_ids].contiguous()
        self.x = x_rows(torch.arange(g.c0, g.c1), device, seed)
        # the row group's whole rows, kept for the oracle check of sampled output rows
        self.rows_ip, self.rows_src, self.rows_alpha = (lip, src, alpha) if keep_rows else (None, None, None)
        note(f"tile ({g.i},{g.j}): {self.graph.nnz} edges, columns [{g.c0}, {g.c1})")

    def sample_rows(self, y_own, owned, k=256, seed=1):
        """Sampled rows of this rank's output for the oracle: (global row ids, local indptr,
        source ids, alpha, X rows of those sources, GPU output rows).  Includes the heaviest and
        the lightest owned row.  Everything is copied to the host."""
        assert self.rows_ip is not None, "shard built with keep_rows=False"
        owned = owned.to(torch.int64)
        ok = torch.nonzero(owned >= 0).flatten()
        if ok.numel() == 0:
            return None
        r0 = self.rcuts[self.grid.i]
        lip = self.rows_ip.cpu()
        rows_local = owned[ok] - r0
        deg = lip[rows_local + 1] - lip[rows_local]
        gen = torch.Generator().manual_seed(seed + self.grid.rank)
        pick = torch.randperm(ok.numel(), generator=gen)[:k]
        pick = torch.unique(torch.cat([pick, torch.argmax(deg).view(1), torch.argmin(deg).view(1)]))
        pos = ok[pick]                       # positions in y_own
        rl = rows_local[pick]
        starts, ends = lip[rl], lip[rl + 1]
        eidx = torch.cat([torch.arange(int(a), int(b)) for a, b in zip(starts, ends)]) \
            if int((ends - starts).sum()) else torch.zeros(0, dtype=torch.int64)
        sub_ip = torch.zeros(rl.numel() + 1, dtype=torch.int64)
        sub_ip[1:] = torch.cumsum(ends - starts, 0)
        src = self.rows_src[eidx.to(self.device)]
        uniq, inv = torch.unique(src, return_inverse=True)
        xs = x_rows(uniq, self.device, self.seed)
        return {"rows": (rl + r0).numpy(), "indptr": sub_ip.numpy(), "indices": inv.cpu().numpy(),
                "alpha": self.rows_alpha[eidx.to(self.device)].cpu().numpy(), "x": xs.cpu().numpy(),
                "y": y_own[pos.to(y_own.device)].cpu().numpy()}
