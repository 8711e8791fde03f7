"""Sequence parallelism for the DiT.

Replaces the reference's xfuser path: ``enable_multi_gpus_inference`` (wan_fantasy_transformer3d_1B.py
:918-923) patches every self-attention with ``usp_attn_forward`` (wan/dist/wan_xfuser.py:72-115), whose
``xFuserLongContextAttention`` runs Ulysses all-to-all (+ ring) attention over a token-sharded residual
stream, and the model all-gathers the head output (1B:1150-1152).

Here, one process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI):

* the residual stream of every CFG row is split into ``world`` contiguous token chunks of
  ``Lc = Lp / world`` tokens (1B:1019 semantics, Lp padded to a multiple of ``world`` at 1B:980);
* heads are split into ``G`` groups (``G`` = the largest common divisor of heads and world) and the
  query rows into ``R = world / G`` parts.  Rank ``r`` owns head group ``r % G`` for query part
  ``r // G``: it receives Q of its head group for the ``G`` chunks of its part and K/V of its head
  group for all chunks (one all-to-all), runs full-sequence attention, and returns O to the chunk
  owners (a second all-to-all).  R = 1 is plain Ulysses (N = 2, 4 with 12 heads); N = 8 gives 4 head
  groups x 2 query halves, the K/V of a group going to both halves (no log-sum-exp merge needed);
* the per-frame vocal attention keeps single-GPU semantics: a local token's frame is its GLOBAL index
  // tokens-per-frame (the reference's SP path regroups them wrongly);
* the head output is all-gathered so every rank holds the full noise prediction and runs the same
  sampler step (bit-identical latents on every rank).

Everything in this module is data movement (torch copies + collectives); the attention itself is the
HIP kernel, called by the transformer.  The exchange is written against torch.distributed only, so
the same code runs under gloo on CPU (tests/test_sp_cpu.py) and RCCL on MI355X.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class SPPlan:
    world: int
    rank: int
    heads: int
    G: int  # head groups
    R: int  # query parts

    @property
    def hg(self) -> int:
        return self.heads // self.G

    @property
    def group(self) -> int:
        return self.rank % self.G

    @property
    def part(self) -> int:
        return self.rank // self.G

    def part_of_chunk(self, r: int) -> int:
        return r // self.G


def make_plan(world: int, rank: int, heads: int) -> SPPlan:
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    G = math.gcd(heads, world)
    return SPPlan(world, rank, heads, G, world // G)


def padded_len(seq_len: int, world: int) -> int:
    """1B:980-981: the token axis is padded up to a multiple of the SP degree."""
    return int(math.ceil(seq_len / world)) * world


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group) -> None:
    """all_to_all_single on flat buffers; gloo cannot move device tensors, so they are staged
    through host memory there (test configuration: several ranks sharing one GPU)."""
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


class Pending:
    """An issued all-to-all and the unpack that runs once it has landed.

    On RCCL the collective runs on ProcessGroupNCCL's own stream; ``wait()`` makes the caller's
    current stream wait for it (no host sync) and then enqueues the unpack copies there, so compute
    queued on the current stream between issue and ``wait()`` overlaps the transfer."""

    def __init__(self, work, finish):
        self.work, self.finish = work, finish

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None
        if self.finish is not None:
            self.finish()
            self.finish = None


def _a2a_async(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group):
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        _a2a(out, inp, out_splits, in_splits, group)  # host-staged: completes here
        return None
    return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=True)


class UlyssesExchange:
    """The two all-to-alls around one sequence-parallel self-attention.

    ``to_heads`` / ``to_tokens`` move all CFG rows in one collective each.  ``to_heads_row`` /
    ``to_tokens_row`` move one CFG row and return a ``Pending``: the transformer issues the three
    rows' Q/K/V exchanges up front and runs row b's attention while rows b+1.. are in flight and row
    b-1's output travels back (comm/compute overlap on separate HIP streams)."""

    def __init__(self, plan: SPPlan, group=None):
        self.plan = plan
        self.group = group

    # tokens -> heads ---------------------------------------------------------------------------
    def to_heads(self, qkv: torch.Tensor, B: int, Lc: int, D: int):
        """qkv: [B*Lc, 3*H*D] (q | k | v, head h at column h*D) of this rank's chunk.
        Returns q [B*Lq, hg*D] (Lq = G*Lc query rows of this rank's part, batch-major) and
        kv [B*Lp, 2*hg*D] (k | v of this rank's head group for the full sequence)."""
        p = self.plan
        N, G, hg = p.world, p.G, p.hg
        H = p.heads
        x = qkv.view(B, Lc, 3, G, hg * D)
        q_el = B * Lc * hg * D
        kv_el = 2 * q_el
        sends, in_splits = [], []
        my_part = p.part_of_chunk(p.rank)
        for j in range(N):
            gj, pj = j % G, j // G
            blk = []
            if pj == my_part:
                blk.append(x[:, :, 0, gj].reshape(-1))
            blk.append(x[:, :, 1:3, gj].reshape(-1))  # [B, Lc, 2, hg*D]
            sends.extend(blk)
            in_splits.append(sum(t.numel() for t in blk))
        send = torch.cat(sends)
        out_splits = []
        for r in range(N):
            out_splits.append((q_el if p.part_of_chunk(r) == p.part else 0) + kv_el)
        recv = torch.empty(sum(out_splits), dtype=qkv.dtype, device=qkv.device)
        _a2a(recv, send, out_splits, in_splits, self.group)
        # unpack: per source rank r, [Q (if r in my part)] [KV]
        qs, kvs = [], []
        off = 0
        for r in range(N):
            if p.part_of_chunk(r) == p.part:
                qs.append(recv[off:off + q_el].view(B, Lc, hg * D))
                off += q_el
            kvs.append(recv[off:off + kv_el].view(B, Lc, 2 * hg * D))
            off += kv_el
        q = torch.stack(qs, 1).reshape(B * len(qs) * Lc, hg * D)        # [B, G*Lc, hg*D]
        kv = torch.stack(kvs, 1).reshape(B * N * Lc, 2 * hg * D)         # [B, Lp, (k|v) hg*D]
        del H
        return q, kv

    # heads -> tokens ---------------------------------------------------------------------------
    def to_tokens(self, o: torch.Tensor, B: int, Lc: int, D: int, out: torch.Tensor) -> torch.Tensor:
        """o: [B*G*Lc, hg*D] attention output of this rank's (part, head group); out: [B*Lc, H*D]
        receives this rank's chunk for all heads."""
        p = self.plan
        N, G, hg = p.world, p.G, p.hg
        el = B * Lc * hg * D
        ov = o.view(B, G, Lc, hg * D)
        sends, in_splits = [], []
        for r in range(N):
            if p.part_of_chunk(r) == p.part:
                sends.append(ov[:, r - p.part * G].reshape(-1))
                in_splits.append(el)
            else:
                in_splits.append(0)
        send = torch.cat(sends)
        out_splits = [el if (j // G) == p.part_of_chunk(p.rank) else 0 for j in range(N)]
        recv = torch.empty(sum(out_splits), dtype=o.dtype, device=o.device)
        _a2a(recv, send, out_splits, in_splits, self.group)
        # sources j with part == my chunk's part, in j order = head group order
        parts = recv.view(G, B, Lc, hg * D)
        out.view(B, Lc, G, hg * D).copy_(parts.permute(1, 2, 0, 3))
        return out

    # one CFG row at a time, asynchronous ----------------------------------------------------------
    def to_heads_row(self, qkv: torch.Tensor, b: int, B: int, Lc: int, D: int,
                     q_dst: torch.Tensor, kv_dst: torch.Tensor) -> Pending:
        """Row b of ``to_heads``: q_dst [B*G*Lc, hg*D] and kv_dst [B*Lp, 2*hg*D] (the layouts
        ``to_heads`` returns) receive row b once the returned Pending is waited on."""
        p = self.plan
        N, G, hg = p.world, p.G, p.hg
        x = qkv.view(B, Lc, 3, G, hg * D)[b]
        q_el = Lc * hg * D
        kv_el = 2 * q_el
        my_part = p.part_of_chunk(p.rank)
        sends, in_splits = [], []
        for j in range(N):
            gj, pj = j % G, j // G
            n = 0
            if pj == my_part:
                sends.append(x[:, 0, gj].reshape(-1))
                n += q_el
            sends.append(x[:, 1:3, gj].reshape(-1))  # [Lc, 2, hg*D]
            in_splits.append(n + kv_el)
        send = torch.cat(sends)
        src_q = [p.part_of_chunk(r) == p.part for r in range(N)]
        out_splits = [(q_el if src_q[r] else 0) + kv_el for r in range(N)]
        recv = torch.empty(sum(out_splits), dtype=qkv.dtype, device=qkv.device)
        work = _a2a_async(recv, send, out_splits, in_splits, self.group)
        Lq = G * Lc

        def finish():
            qv = q_dst.view(B, Lq, hg * D)[b]
            kvv = kv_dst.view(B, N * Lc, 2 * hg * D)[b]
            off, qi = 0, 0
            for r in range(N):
                if src_q[r]:
                    qv[qi * Lc:(qi + 1) * Lc].copy_(recv[off:off + q_el].view(Lc, hg * D))
                    qi += 1
                    off += q_el
                kvv[r * Lc:(r + 1) * Lc].copy_(recv[off:off + kv_el].view(Lc, 2 * hg * D))
                off += kv_el

        return Pending(work, finish)

    def to_tokens_row(self, o: torch.Tensor, b: int, B: int, Lc: int, D: int, out: torch.Tensor) -> Pending:
        """Row b of ``to_tokens``: o [B*G*Lc, hg*D]; out [B*Lc, H*D] receives row b on wait()."""
        p = self.plan
        N, G, hg = p.world, p.G, p.hg
        el = Lc * hg * D
        ov = o.view(B, G, Lc, hg * D)[b]
        sends, in_splits = [], []
        for r in range(N):
            if p.part_of_chunk(r) == p.part:
                sends.append(ov[r - p.part * G].reshape(-1))
                in_splits.append(el)
            else:
                in_splits.append(0)
        send = torch.cat(sends)
        out_splits = [el if (j // G) == p.part_of_chunk(p.rank) else 0 for j in range(N)]
        recv = torch.empty(sum(out_splits), dtype=o.dtype, device=o.device)
        work = _a2a_async(recv, send, out_splits, in_splits, self.group)

        def finish():
            out.view(B, Lc, G, hg * D)[b].copy_(recv.view(G, Lc, hg * D).permute(1, 0, 2))

        return Pending(work, finish)


def all_gather_slots(buf: torch.Tensor, rank: int, group=None) -> Pending:
    """Window parallelism: buf [world, S]; row ``rank`` holds this rank's noise
    prediction of one window, every row is filled on every rank once the Pending is waited on."""
    mine = buf[rank:rank + 1]  # [1, S]: the output is gathered as [world, S]
    if dist.get_backend(group) == "gloo":
        if buf.is_cuda:  # host-staged (several ranks sharing one GPU in tests)
            o = torch.empty(buf.shape, dtype=buf.dtype)
            dist.all_gather_into_tensor(o, mine.cpu().contiguous(), group=group)
            buf.copy_(o)
        else:
            dist.all_gather_into_tensor(buf, mine.clone(), group=group)
        return Pending(None, None)
    return Pending(dist.all_gather_into_tensor(buf, mine, group=group, async_op=True), None)


def gather_tokens(local: torch.Tensor, B: int, Lc: int, world: int, group=None) -> torch.Tensor:
    """[B*Lc, C] chunk of every rank -> [B*Lp, C] (batch-major), on every rank (1B:1150-1152)."""
    C = local.shape[1]
    if local.is_cuda and dist.get_backend(group) == "gloo":
        buf = torch.empty(world * B * Lc, C, dtype=local.dtype)
        dist.all_gather_into_tensor(buf, local.cpu().contiguous(), group=group)
        buf = buf.to(local.device)
    else:
        buf = torch.empty(world * B * Lc, C, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(buf, local.contiguous(), group=group)
    return buf.view(world, B, Lc, C).permute(1, 0, 2, 3).reshape(B * world * Lc, C)


def local_segments(B: int, Lc: int, kv_len: int):
    """cross-attention segments (text / image) of the local chunk: [q_row0, q_len, kv_row0, kv_len]."""
    return [[b * Lc, Lc, b * kv_len, kv_len] for b in range(B)]


def vocal_segments(B: int, S: int, Lc: int, rank: int, n_frames: int, nper: int):
    """Per-frame vocal attention segments for this rank's chunk with single-GPU frame grouping:
    global token t < S belongs to frame t // (S / n_frames) (1B:575-586 on the unsharded sequence of S
    tokens); SP pad tokens past S (queries whose outputs are never read) join the last frame's segment."""
    G = S // n_frames
    t0, t1 = rank * Lc, (rank + 1) * Lc
    segs = []
    for b in range(B):
        for f in range(min(t0 // G, n_frames - 1), min((t1 - 1) // G, n_frames - 1) + 1):
            a = max(f * G, t0)
            e = min((f + 1) * G, t1) if f < n_frames - 1 else t1
            if e > a:
                segs.append([b * Lc + a - t0, e - a, (b * n_frames + f) * nper, nper])
    return segs
