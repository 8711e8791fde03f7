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

This module holds the layout and the transfers (torch.distributed point-to-point: RCCL on MI355X, gloo on
CPU in tests/test_sp_cpu.py); the pack (RMSNorm + RoPE writing send slabs), the attention (writing its
output by row map) and the O-projection (reading column panels) are HIP kernels called by the transformer,
so no copy pass runs on the way in or out.
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


def _panel_slack_rows(device) -> int:
    """Rows the column-panel O-projection may read past its last panel (sa_gemm_panel_slack_rows).  Only a GPU
    exchange runs that GEMM: on the CPU (the gloo protocol tests) no slack is needed and the HIP library is not
    loaded."""
    if torch.device(device).type != "cuda":
        return 0
    from . import _lib
    return int(_lib.lib().sa_gemm_panel_slack_rows())


def padded_len(seq_len: int, world: int) -> int:
    """1B:980-981: the token axis is padded up to a multiple of the SP degree."""
    return int(math.ceil(seq_len / world)) * world


class Pending:
    """Issued point-to-point transfers and the host-staged copies (gloo only) that finish them.

    On RCCL the transfers run on ProcessGroupNCCL's own stream; ``wait()`` makes the caller's current
    stream wait for them (no host sync), so compute queued on the current stream between issue and
    ``wait()`` overlaps the transfer."""

    def __init__(self, works, finish=None, keep=None):
        self.works, self.finish, self.keep = works, finish, keep

    def wait(self):
        for w in self.works or ():
            w.wait()
        self.works = None
        if self.finish is not None:
            self.finish()
            self.finish = None
        self.keep = None


def _p2p(sends, recvs, group):
    """sends / recvs: lists of (contiguous tensor, peer rank inside ``group``).  RCCL: one coalesced group of sends and
    receives landing in place (a peer may be this rank itself: loopback, matched in order like any peer's).  gloo
    cannot move device tensors, so there (several ranks sharing one GPU in the tests) they are staged through host
    memory and the device receive views are filled on wait(); gloo has no pair to the own rank, so loopback
    transfers are matched in order and copied locally."""
    if not sends and not recvs:
        return Pending(None)
    t0 = (sends or recvs)[0][0]
    if dist.get_backend(group) != "gloo":
        ops = [dist.P2POp(dist.isend, t, group=group, group_peer=peer) for t, peer in sends]
        ops += [dist.P2POp(dist.irecv, t, group=group, group_peer=peer) for t, peer in recvs]
        return Pending(dist.batch_isend_irecv(ops), keep=(sends, recvs))
    me = dist.get_rank(group)
    self_s = [t for t, peer in sends if peer == me]
    self_r = [t for t, peer in recvs if peer == me]
    if len(self_s) != len(self_r):
        raise RuntimeError(f"loopback: {len(self_s)} sends to this rank but {len(self_r)} receives from it")
    for s_, r_ in zip(self_s, self_r):
        r_.copy_(s_)
    sends = [(t, peer) for t, peer in sends if peer != me]
    recvs = [(t, peer) for t, peer in recvs if peer != me]
    staged = t0.is_cuda
    works, keep, back = [], [], []
    for t, peer in sends:
        h = t.cpu() if staged else t
        keep.append(h)
        works.append(dist.isend(h, group=group, group_dst=peer))
    for t, peer in recvs:
        h = torch.empty(t.shape, dtype=t.dtype) if staged else t
        keep.append(h)
        works.append(dist.irecv(h, group=group, group_src=peer))
        if staged:
            back.append((t, h))

    def finish():
        for t, h in back:
            t.copy_(h)

    return Pending(works, finish if back else None, keep)


class UlyssesExchange:
    """The data layout and the point-to-point transfers around one sequence-parallel self-attention
    (usp_attn_forward, wan/dist/wan_xfuser.py:72-115), for B CFG rows of Lc tokens per rank.

    There is no pack or unpack pass: every tensor lands where its consumer reads it.
      * ``q`` [B*Lq, hg*D] (rows b*Lq + j*Lc + t: token t of chunk j of this rank's query part) and ``kv``
        [B*Lp, 2*hg*D] (rows b*Lp + r*Lc + t, k | v) are the attention inputs; this rank's own chunk is
        written into them by ``ops.qkv_pack`` (through ``table``), the other chunks arrive into them;
      * ``sq[d]`` [B, Lc, hg*D] and ``skv[d]`` [B, Lc, 2*hg*D] are the send slabs of remote destination d of this
        rank's query part, also written by ``ops.qkv_pack``; the K/V of head group j goes to the group's rank of every
        query part from the one slab of this part (``kv_source(j)``: written once, sent R times);
      * ``obuf`` [2*G*B*Lc, hg*D]: the attention writes query chunk j's head outputs to rows (j*B + b)*Lc + t
        of the first half (the send slab of chunk j's owner) -- except this rank's own chunk, which goes to
        the second half, ``pan``, whose panel j (rows j*B*Lc ..) receives head group j of this rank's tokens
        from the other ranks of the query part: ``pan`` is the O-projection's input in column panels
        (``ops.linear(..., a_panels=(hg*D, B*Lc*hg*D))``).  ``omap`` is that attention output row map.

    ``loopback=True`` sends this rank's own chunk through the transport as well (its Q/K/V through send slabs of
    its own, its head outputs through the first half of ``obuf``), a point-to-point transfer to itself: at degree 1
    on RCCL that runs every send / receive of the exchange on the GPU the box has, with a bit-identical result."""

    def __init__(self, plan: SPPlan, B: int, Lc: int, D: int, device, group=None, dtype=torch.bfloat16,
                 loopback=False):
        self.plan, self.group, self.B, self.Lc, self.D = plan, group, B, Lc, D
        self.loopback = bool(loopback)
        p = plan
        N, G, g = p.world, p.G, p.group
        self.hgd = hgd = p.hg * D
        self.Lq, self.Lp = G * Lc, N * Lc
        self.q = torch.empty(B * self.Lq, hgd, device=device, dtype=dtype)
        self.kv = torch.empty(B * self.Lp, 2 * hgd, device=device, dtype=dtype)
        # + slack rows: the O-projection's last tile reads up to its tile height past the last panel
        # (sa_gemm_bf16_panels; the buffer range check does not cover the panel offset).  The slack comes from
        # the library (sa_gemm_panel_slack_rows = the tallest GEMM tile), so a taller tile cannot outgrow it.
        # On the per-row-stream path (transformer._sp_layer_rows) row b's O-projection tail tile also reads
        # into row b+1's panel region while another stream may be writing it: benign, those rows' products are
        # discarded (never stored), only their bytes are fetched.
        self.obuf = torch.empty(2 * G * B * Lc + _panel_slack_rows(device), hgd, device=device, dtype=dtype)
        self.pan = self.obuf[G * B * Lc:2 * G * B * Lc]
        self.remote = [d for d in range(N) if d != p.rank or self.loopback]
        mine = [d for d in self.remote if d // G == p.part]  # destinations of this query part
        self.sq = {d: torch.empty(B, Lc, hgd, device=device, dtype=dtype) for d in mine}
        self.skv = {d: torch.empty(B, Lc, 2 * hgd, device=device, dtype=dtype) for d in mine}
        qv = self.q.view(B, self.Lq, hgd)
        kvv = self.kv.view(B, self.Lp, 2 * hgd)
        self.slabs = {d: (self.sq[d], self.skv[d]) for d in mine}
        if not self.loopback:
            self.slabs[p.rank] = (qv[:, g * Lc:(g + 1) * Lc], kvv[:, p.rank * Lc:(p.rank + 1) * Lc])
        rows = []
        for d in range(N):
            qd, kd = self.slabs.get(d, (None, None))  # other query parts' rows: not read by the pack
            rows.append(([0, 0, 0] if qd is None else [qd.data_ptr(), qd.stride(1), qd.stride(0)]) +
                        ([0, 0, 0] if kd is None else [kd.data_ptr(), kd.stride(1), kd.stride(0)]))
        self.table = torch.tensor(rows, dtype=torch.int64).to(device)
        j = torch.arange(G).view(1, G, 1)
        b = torch.arange(B).view(B, 1, 1)
        t = torch.arange(Lc).view(1, 1, Lc)
        own = (j == g).to(torch.int64) * (0 if self.loopback else 1)  # own chunk straight into its panel
        omap = own * (G * B * Lc) + (j * B + b) * Lc + t  # [B, G, Lc] = q row order
        self.omap = omap.reshape(-1).to(torch.int32).to(device)

    def kv_source(self, j):
        """the k | v slab [B, Lc, 2*hg*D] of head group j that the pack wrote (this query part's destination of the
        group), sent to the group's rank in every query part"""
        d = self.plan.part * self.plan.G + j
        return self.slabs[d][1]

    def heads(self, rows) -> Pending:
        """Q/K/V of CFG rows ``rows`` to the ranks that attend over them (after ``ops.qkv_pack``)."""
        p = self.plan
        G, Lc, Lq, Lp = p.G, self.Lc, self.Lq, self.Lp
        sends, recvs = [], []
        for b in rows:
            for d in self.remote:
                if d in self.sq:
                    sends.append((self.sq[d][b], d))
                sends.append((self.kv_source(d % G)[b], d))
            for r in self.remote:
                if r // G == p.part:
                    q0 = b * Lq + (r % G) * Lc
                    recvs.append((self.q[q0:q0 + Lc], r))
                recvs.append((self.kv[b * Lp + r * Lc:b * Lp + (r + 1) * Lc], r))
        return _p2p(sends, recvs, self.group)

    def tokens(self, rows) -> Pending:
        """Head outputs of CFG rows ``rows`` back to the owners of their tokens (after the attention)."""
        p = self.plan
        G, B, Lc = p.G, self.B, self.Lc
        sends, recvs = [], []
        for b in rows:
            for j in range(G):
                if j != p.group or self.loopback:
                    r0 = (j * B + b) * Lc
                    sends.append((self.obuf[r0:r0 + Lc], p.part * G + j))
            for j in range(G):
                if j != p.group or self.loopback:
                    r0 = (j * B + b) * Lc
                    recvs.append((self.pan[r0:r0 + Lc], p.part * G + j))
        return _p2p(sends, recvs, self.group)

    def panels(self, rows=None):
        """(first panel [M, hg*D], (panel_cols, panel_stride)) of the O-projection input for CFG rows
        ``rows`` (a range; None = all)"""
        B, Lc = self.B, self.Lc
        b0, nb = (0, B) if rows is None else (rows.start, len(rows))
        return self.pan[b0 * Lc:(b0 + nb) * Lc], (self.hgd, B * Lc * self.hgd)


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
    return Pending([dist.all_gather_into_tensor(buf, mine, group=group, async_op=True)], None)


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
