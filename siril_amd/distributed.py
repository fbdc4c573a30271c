"""Multi-GPU rejection stack: pixel-row bands, one process per GPU.

Every output pixel is a function of its own N-sample column only, so the
exact decomposition is by rows (finding F3): rank r stacks the
rows [y0_r, y1_r) of all N frames -- the same row blocks Siril hands to its
OpenMP threads (stack_compute_parallel_blocks, median_and_mean.c:295-356) --
with no exchange during compute.  Afterwards:
  * the output bands are all-gathered (RCCL over xGMI with backend "nccl"),
  * the low/high rejection totals are all-reduced.
Frame sharding + partial-sum all-reduce would only be exact for the
no-rejection mean; sigma / Winsorized / median need whole columns.

Frame-sharded input (BASELINE config 4's wording: each GPU holds N/world
whole frames) is handled by `stack_frame_sharded`:
  * the unweighted no-rejection mean is the one case the north star's
    partial-sum / partial-count all-reduce computes exactly: every rank
    accumulates per pixel the f64 sum and the count of its present samples
    (sgpu_mean_partial_device), both are all-reduced, and the mean is
    finished on every rank (sgpu_mean_finish_device);
  * every other method needs whole columns, so the shards are transposed to
    row bands with one all-to-all (each rank sends rows band_d of its frames
    to rank d: (world-1)/world of its shard crosses xGMI) and the row-band
    stack above runs unchanged.

Normalization of frame-sharded input (`normalization_frame_sharded`): each
frame's estimators (median, MAD, IKSS location / scale of the whole frame,
statistics_float.c:281-480) depend on that frame only, and a frame shard
holds its frames whole, so every rank runs the estimator kernels on its own
frames with no exchange; the per-frame tables (N x 6 numbers) are
all-gathered and every rank derives the same factors against the reference
frame (compute_factors_from_estimators, normalization.c:150-185).  This runs
before the all-to-all, on the layout the frames are loaded in, so no
histogram ever needs reducing across ranks.

With args.output_norm the gathered image gets the reference's whole-image
norm_to_0_1_range (median_and_mean.c:557-582, applied after the stack at
:1774-1775): min / max over the full image, so it runs after the gather, on
every rank, never per band.

The per-band compute is `Context.stack_device` by default; tests inject a
CPU compute function to check the decomposition with the gloo backend.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple


def row_bands(height: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced row bands [y0, y1) covering [0, height)."""
    base, extra = divmod(height, world)
    bands, y = [], 0
    for r in range(world):
        h = base + (1 if r < extra else 0)
        bands.append((y, y + h))
        y += h
    return bands


def stack_row_band(frames_band, args, method, ctx=None, compute: Optional[Callable] = None):
    """Stack one band; returns (out [rows, W] float32 tensor, counts [2] int64 tensor)."""
    import torch
    if compute is not None:
        return compute(frames_band, args, method)
    out, _, _, counts = ctx.stack_device(frames_band, args, method)
    return out, counts


def _output_norm(full, args, ctx=None, post: Optional[Callable] = None):
    """norm_to_0_1_range of the whole gathered image when args.output_norm
    (32-bit output, median_and_mean.c:1774-1775); `post` replaces the HIP
    pass in CPU tests."""
    if not getattr(args, "output_norm", False):
        return full
    if post is not None:
        return post(full)
    return ctx.norm_to_0_1_range_device(full.contiguous())


def stack_distributed(frames_band, height: int, args, method: int = 0, ctx=None,
                      compute: Optional[Callable] = None, group=None, post: Optional[Callable] = None):
    """Collective over the default process group.  `frames_band` holds this
    rank's rows [y0, y1) of every frame ([N, y1-y0, W], on this rank's device
    for backend nccl).  Returns (full image [height, W] on every rank,
    (rejected_low, rejected_high) totals)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    bands = row_bands(height, world)
    y0, y1 = bands[rank]
    n, rows, W = frames_band.shape
    if rows != y1 - y0:
        raise ValueError(f"rank {rank} holds {rows} rows, band is {y1 - y0}")
    out, counts = stack_row_band(frames_band, args, method, ctx, compute)
    # pad every band to the largest one so all_gather sees equal shapes
    hmax = max(b1 - b0 for b0, b1 in bands)
    pad = torch.zeros((hmax, W), dtype=out.dtype, device=out.device)
    pad[:rows] = out
    gathered = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad, group=group)
    full = torch.cat([g[: b1 - b0] for g, (b0, b1) in zip(gathered, bands)], dim=0)
    counts = counts.to(torch.int64).clone()
    dist.all_reduce(counts, group=group)
    full = _output_norm(full, args, ctx, post)
    return full, (int(counts[0]), int(counts[1]))


def frame_shards(nframes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous balanced frame ranges [f0, f1) (frames keep their order)."""
    return row_bands(nframes, world)


def _transport_view(t):
    """RCCL has no 16-bit integer type: move 16-bit samples as float16 bits."""
    import torch
    if t.dtype in (torch.int16, getattr(torch, "uint16", torch.int16)):
        return t.view(torch.float16)
    return t


# Largest piece one rank hands to one peer in one collective.  RCCL's
# all_to_all_single corrupts pieces past 2 GiB (measured on the MI355X box,
# world-1 nccl, profiles/r06b_fs_check.log: 1 Gi-element = 4 GiB pieces
# arrive wrong; 96 MB point-to-point pieces arrive right), so every exchange
# below is cut into row sub-chunks whose pieces stay under this bound.
MAX_PIECE_BYTES = 1 << 30
# ... and any one peer's piece under this (at 8 GPUs config 4's pieces are
# 600 MB / sub-chunk; the failures seen were pieces of 2.4 GB and more)
MAX_PEER_PIECE_BYTES = 1 << 28
# At world 1 the "exchange" is a self-copy of the whole shard, which RCCL got
# wrong at these sizes (profiles/r06b_fs_check.log; one step of the capped
# unpipelined path still differed, profiles/r06c_fs_sigma400_p0.json): the
# shard IS the band, so world 1 skips the collective unless a test or the
# bench asks to exercise RCCL on one GPU.
COLLECTIVE_AT_WORLD1 = False


def _min_subchunks(n_r: int, bands, W: int, itemsize: int, nframes: int, rank: int) -> int:
    """Fewest row sub-chunks that keep what rank `rank` sends and what it
    receives in one collective under MAX_PIECE_BYTES, and every single
    peer's piece under MAX_PEER_PIECE_BYTES (whether RCCL's limit is per
    piece or per call was not isolated: both are bounded)."""
    H = bands[-1][1]
    y0, y1 = bands[rank]
    world = len(bands)
    nmax = -(-nframes // world)                          # the largest frame shard
    hmax = max(b1 - b0 for b0, b1 in bands)
    send = n_r * H * W * itemsize                        # all my frames' rows, to every band
    recv = nframes * (y1 - y0) * W * itemsize            # my band of every frame
    piece = max(n_r * hmax, nmax * (y1 - y0)) * W * itemsize
    return max(1, -(-max(send, recv, 1) // MAX_PIECE_BYTES), -(-piece // MAX_PEER_PIECE_BYTES))


def transpose_frames_to_bands(frames_shard, nframes: int, group=None, mode: str = "all_to_all"):
    """All-to-all from frame shards to row bands.  Rank r holds frames
    frame_shards(nframes, world)[r] whole ([n_r, H, W]); returns this rank's
    rows row_bands(H, world)[r] of all nframes frames ([nframes, h_r, W], in
    frame order).

    mode "all_to_all" (default): one `all_to_all_single` with a whole
    contiguous piece per peer.  The shard is first laid out band-major (one
    HBM copy of the shard: the rows of band p of all n_r frames become one
    contiguous piece, at HBM speed, far above a link's ~150 GB/s), and what
    arrives from peer p -- its frames' rows of this band, frame-major -- is
    already in place: shards are contiguous and ascending, so the received
    pieces concatenate to [nframes, h_r, W] with no unpack.  Every rank joins
    the one collective (an empty band or an empty shard is a zero-sized
    piece), so RCCL sees one grouped exchange of world pieces per rank
    instead of n_r x (world - 1) point-to-point operations.

    mode "p2p": no staging copy; every (frame, band) piece goes straight
    from the shard to the peer's output as one point-to-point transfer of a
    batched send / receive (n_r x (world - 1) sends per rank).  RCCL wants
    every rank of the group in the first batched point-to-point call, so
    this mode refuses layouts where a rank would have nothing to send or
    receive (nframes < world or H < world); the all-to-all takes those."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_r, H, W = frames_shard.shape
    shards = frame_shards(nframes, world)
    if n_r != shards[rank][1] - shards[rank][0]:
        raise ValueError(f"rank {rank} holds {n_r} frames, shard is {shards[rank]}")
    if frames_shard.stride(2) != 1 or frames_shard.stride(1) != W:
        raise ValueError("frame rows must be contiguous")
    bands = row_bands(H, world)
    src = _transport_view(frames_shard)
    y0r, y1r = bands[rank]
    hr = y1r - y0r
    if world == 1 and not COLLECTIVE_AT_WORLD1:
        return frames_shard                       # the shard is the band
    if mode == "all_to_all":
        # pieces past MAX_PIECE_BYTES: the exchange in row sub-chunks, each
        # one received whole-column and copied into its rows of the band
        # (every rank computes the same count from the shared layout)
        kmin = max(_min_subchunks(b - a, bands, W, src.element_size(), nframes, r)
                   for r, (a, b) in enumerate(frame_shards(nframes, world)))
        if kmin > 1:
            out = torch.empty((nframes, hr, W), dtype=src.dtype, device=src.device)
            subs = [sub_bands(b, kmin) for b in bands]
            for k in range(kmin):
                ssz = [n_r * (subs[p][k][1] - subs[p][k][0]) * W for p in range(world)]
                b0, b1 = subs[rank][k]
                rsz = [(f1 - f0) * (b1 - b0) * W for f0, f1 in shards]
                send = torch.empty(sum(ssz), dtype=src.dtype, device=src.device)
                o = 0
                for p in range(world):
                    a0, a1 = subs[p][k]
                    if ssz[p]:
                        send[o:o + ssz[p]].view(n_r, a1 - a0, W).copy_(src[:, a0:a1])
                    o += ssz[p]
                recv = torch.empty(sum(rsz), dtype=src.dtype, device=src.device)
                dist.all_to_all_single(recv, send, rsz, ssz, group=group)
                if b1 > b0:
                    out[:, b0 - y0r:b1 - y0r].copy_(recv.view(nframes, b1 - b0, W))
            return out.view(frames_shard.dtype)
        if H % world == 0:            # equal bands: the band-major layout is one strided copy
            send = src.reshape(n_r, world, H // world, W).transpose(0, 1).contiguous().view(-1)
        else:
            send = torch.cat([src[:, y0:y1].reshape(-1) for y0, y1 in bands])
        recv = torch.empty(nframes * hr * W, dtype=src.dtype, device=src.device)
        dist.all_to_all_single(recv, send, [(f1 - f0) * hr * W for f0, f1 in shards],
                               [n_r * (y1 - y0) * W for y0, y1 in bands], group=group)
        return recv.view(nframes, hr, W).view(frames_shard.dtype)
    if mode != "p2p":
        raise ValueError(f"unknown transpose mode {mode!r}")
    if world > 1 and (nframes < world or H < world):
        raise ValueError("p2p transpose needs a frame and a row per rank; use mode='all_to_all'")
    recv = torch.empty((nframes, hr, W), dtype=src.dtype, device=src.device)
    ops = []
    for peer in range(world):
        if peer == rank:
            continue
        y0, y1 = bands[peer]
        if y1 > y0:                                  # my frames' rows of the peer's band
            for f in range(n_r):
                ops.append(dist.P2POp(dist.isend, src[f, y0:y1], peer, group))
        f0, f1 = shards[peer]
        if hr > 0:                                   # the peer's frames' rows of my band
            for f in range(f0, f1):
                ops.append(dist.P2POp(dist.irecv, recv[f], peer, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    f0, f1 = shards[rank]
    recv[f0:f1].copy_(src[:, y0r:y1r])
    return recv.view(frames_shard.dtype)


def sub_bands(band: Tuple[int, int], k: int) -> List[Tuple[int, int]]:
    """Split the row band [y0, y1) into k contiguous balanced sub-chunks
    (absolute rows; empty ones when the band has fewer than k rows)."""
    y0, y1 = band
    return [(y0 + a, y0 + b) for a, b in row_bands(y1 - y0, k)]


def sub_bands_lead(band: Tuple[int, int], k: int) -> List[Tuple[int, int]]:
    """Split [y0, y1) into k contiguous sub-chunks, the first one half the
    size of the others (weights 1, 2, 2, ...): the pipeline's first exchange
    is the only one nothing hides, so it moves the least."""
    y0, y1 = band
    n = y1 - y0
    if k <= 1:
        return [(y0, y1)]
    tot = 2 * k - 1
    cuts = [y0 + (n * (2 * i - 1) + tot - 1) // tot if i else y0 for i in range(k)] + [y1]
    cuts = [min(max(c, y0), y1) for c in cuts]
    return [(cuts[i], cuts[i + 1]) for i in range(k)]


def _gather_bands(out, counts, height: int, args, ctx=None, group=None, post: Optional[Callable] = None):
    """All-gather of the output bands and all-reduce of the rejection totals
    (the tail of stack_distributed)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bands = row_bands(height, world)
    rows, W = out.shape
    hmax = max(b1 - b0 for b0, b1 in bands)
    pad = torch.zeros((hmax, W), dtype=out.dtype, device=out.device)
    pad[:rows] = out
    gathered = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(gathered, pad, group=group)
    full = torch.cat([g[: b1 - b0] for g, (b0, b1) in zip(gathered, bands)], dim=0)
    counts = counts.to(torch.int64).clone()
    dist.all_reduce(counts, group=group)
    full = _output_norm(full, args, ctx, post)
    return full, (int(counts[0]), int(counts[1]))


def stack_frame_sharded_pipelined(frames_shard, nframes: int, args, method: int = 0, ctx=None,
                                  compute: Optional[Callable] = None, group=None,
                                  post: Optional[Callable] = None, subchunks: int = 4, stats: Optional[dict] = None,
                                  ctxs=None, lead: bool = True):
    """Rejection stack of frame-sharded input with the transpose pipelined
    under the stack (BASELINE config 4: N frames sharded by frame over the
    GPUs; reference decomposition: row blocks, median_and_mean.c:295-356).

    Rank r's row band is cut into `subchunks` row sub-chunks.  For sub-chunk
    k every rank stages its frames' rows of every peer's k-th sub-chunk into
    one contiguous send piece (1/subchunks of the shard: no band-major copy
    of the whole shard up front) and joins one `all_to_all_single`; what
    arrives -- the k-th sub-chunk of its band, frame-major from each peer in
    shard order -- is [nframes, h_k, W] with no unpack, and is stacked at
    once into rows of the output band.  On CUDA the staging copy and the
    collective of sub-chunk k+1 are issued from a side stream before the
    stack of sub-chunk k is queued on the current stream, so RCCL moves
    k+1 over xGMI while the stack kernels run k; the current stream waits
    only for the collective it consumes.  With gloo (CPU tests) the same
    sequence runs, the asynchronous collective overlapping the CPU compute.
    Then the output bands are all-gathered and the totals all-reduced, as in
    stack_distributed.  Bit-identical to the unpipelined path: every pixel is
    still a function of its own whole column.

    `ctxs` (CUDA, optional): two or more Contexts; sub-chunk k is stacked on
    ctxs[k % len] on a stream of its own, so one sub-chunk's last waves and
    deferred-pixel tail run under the next one's start (each Context has its
    own workspace, so the launches never share buffers).  The stacks of one
    sub-chunk alone pay that tail in full.

    `lead`: the first sub-chunk half the size of the others (sub_bands_lead):
    its exchange is the pipeline's fill, exposed in full; one more sub-chunk
    is taken when the cap on a collective's bytes requires it.

    `stats`, when given, receives per-sub-chunk timing events on CUDA
    ("events": [(a2a_start, stack_start, stack_end)]) for bench.py."""
    import contextlib
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_r, H, W = frames_shard.shape
    shards = frame_shards(nframes, world)
    if n_r != shards[rank][1] - shards[rank][0]:
        raise ValueError(f"rank {rank} holds {n_r} frames, shard is {shards[rank]}")
    if frames_shard.stride(2) != 1 or frames_shard.stride(1) != W:
        raise ValueError("frame rows must be contiguous")
    bands = row_bands(H, world)
    dev = frames_shard.device
    cuda = frames_shard.is_cuda
    if ctx is None and ctxs:
        ctx = ctxs[0]
    if world == 1 and not COLLECTIVE_AT_WORLD1:
        # the shard is the band: stack it in place, no exchange
        out = torch.empty((H, W), dtype=torch.float32, device=dev)
        counts = torch.zeros(2, dtype=torch.int64, device=dev)
        if compute is not None:
            o, c = compute(frames_shard, args, method)
            out[:] = o
            counts += c.to(torch.int64).to(dev)
        else:
            ctx.stack_device(frames_shard, args, method, out=out, counts=counts)
        if stats is not None:
            stats["events"] = []
            stats["subchunks"] = 0
        return _gather_bands(out, counts, H, args, ctx, group, post)
    # at least enough sub-chunks to keep every piece under MAX_PIECE_BYTES
    # (the same count on every rank: it is computed from the shared layout)
    kmin = max(_min_subchunks(b - a, bands, W, frames_shard.element_size(), nframes, r)
               for r, (a, b) in enumerate(shards))
    K = max(1, int(subchunks), kmin)
    split = sub_bands
    if lead and K > 1:
        # the largest lead-split piece is 2 / (2K - 1) of the band: at least
        # as many sub-chunks as that needs under the cap (kmin equal ones)
        while K < 2 * kmin and 2 * kmin > 2 * K - 1:
            K += 1
        split = sub_bands_lead
    sb = [split(b, K) for b in bands]                    # sb[peer][k] = rows of the peer's k-th sub-chunk
    src = _transport_view(frames_shard)
    y0r, y1r = bands[rank]
    out = torch.empty((y1r - y0r, W), dtype=torch.float32, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    # buffers allocated up front on the current stream: one shard of send
    # pieces, one band of received columns (views per sub-chunk)
    send_sz = [[n_r * (b1 - b0) * W for (b0, b1) in (sb[p][k] for p in range(world))] for k in range(K)]
    recv_sz = [[(f1 - f0) * (sb[rank][k][1] - sb[rank][k][0]) * W for (f0, f1) in shards] for k in range(K)]
    send = torch.empty(sum(map(sum, send_sz)), dtype=src.dtype, device=dev)
    recv = torch.empty(nframes * (y1r - y0r) * W, dtype=src.dtype, device=dev)
    soff = [0]
    for k in range(K):
        soff.append(soff[-1] + sum(send_sz[k]))
    roff = [0]
    for k in range(K):
        roff.append(roff[-1] + sum(recv_sz[k]))
    main = torch.cuda.current_stream(dev) if cuda else None
    side = torch.cuda.Stream(dev) if cuda else None
    if cuda:
        side.wait_stream(main)                            # the shard and the buffers are ready
    # stack lanes: (context, stream, counts) per lane; lane 0 is the current stream
    multi = cuda and compute is None and ctxs is not None and len(ctxs) > 1
    lanes = [(ctx, main, counts)]
    if multi:
        for c in ctxs[1:]:
            cnt = torch.zeros(2, dtype=torch.int64, device=dev)   # zeroed on the current stream ...
            st = torch.cuda.Stream(dev)
            st.wait_stream(main)                                    # ... before the lane's first use
            lanes.append((c, st, cnt))
    ev = [] if (stats is not None and cuda) else None
    works = [None] * K

    def issue(k):
        with (torch.cuda.stream(side) if cuda else contextlib.nullcontext()):
            e0 = None
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(side)
            o = soff[k]
            for p in range(world):
                b0, b1 = sb[p][k]
                m = send_sz[k][p]
                if m:
                    send[o:o + m].view(n_r, b1 - b0, W).copy_(src[:, b0:b1])
                o += m
            works[k] = (dist.all_to_all_single(recv[roff[k]:roff[k + 1]], send[soff[k]:soff[k + 1]],
                                               recv_sz[k], send_sz[k], group=group, async_op=True), e0)

    issue(0)
    for k in range(K):
        if k + 1 < K:
            issue(k + 1)
        w, e0 = works[k]
        c_k, st_k, cnt_k = lanes[k % len(lanes)]
        with (torch.cuda.stream(st_k) if cuda else contextlib.nullcontext()):
            w.wait()                   # nccl: this lane's stream waits for the collective
        works[k] = None
        b0, b1 = sb[rank][k]
        if b1 == b0:
            continue
        band = recv[roff[k]:roff[k + 1]].view(nframes, b1 - b0, W).view(frames_shard.dtype)
        e1 = e2 = None
        if ev is not None:
            e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
            e1.record(st_k)
        if compute is not None:
            o_k, cc = compute(band, args, method)
            out[b0 - y0r:b1 - y0r] = o_k
            counts += cc.to(torch.int64).to(dev)
        else:
            c_k.stack_device(band, args, method, out=out[b0 - y0r:b1 - y0r], counts=cnt_k, stream=st_k)
        if ev is not None:
            e2.record(st_k)
            ev.append((e0, e1, e2))
    for _, st, cnt in lanes[1:]:      # join the other lanes into the current stream
        main.wait_stream(st)
        counts += cnt
    if stats is not None:
        stats["events"] = ev
        stats["subchunks"] = K
    return _gather_bands(out, counts, H, args, ctx, group, post)


def partial_sums_exact(count, amin, amax):
    """The exactness condition of the frame-sharded partial sums (torch):
    True where every order of the f64 additions of the `count` present
    samples (|x| in [amin, amax]) gives the same double -- all on the grid of
    ulp(amin), every partial sum within 2^53 of it:
    ceil(log2 count) + e(amax) - e(amin) + 24 <= 53 (stack_partial.hip)."""
    import torch

    def fexp(a):
        e = (a.contiguous().view(torch.int32) >> 23) & 0xFF
        return torch.where(e == 0, torch.full_like(e, -126), e - 127)
    c = count.to(torch.int64)
    cl = torch.ceil(torch.log2(torch.clamp(c, min=1).to(torch.float64))).to(torch.int64)
    return (c <= 1) | (cl + fexp(amax) - fexp(amin) + 24 <= 53)


def _sequential_means(cols, output_norm: bool):
    """Mean of the non-zero samples of each column of cols [N, k] (float32),
    summed in f64 in frame order (median_and_mean.c:1083-1097, the oracle's
    sequential order), clamped to [0, 1] unless output_norm."""
    import torch
    acc = torch.zeros(cols.shape[1], dtype=torch.float64, device=cols.device)
    cnt = torch.zeros(cols.shape[1], dtype=torch.int64, device=cols.device)
    for f in range(cols.shape[0]):
        x = cols[f].to(torch.float64)
        nz = x != 0
        acc = torch.where(nz, acc + x, acc)
        cnt += nz
    m = torch.where(cnt > 0, acc / torch.clamp(cnt, min=1).to(torch.float64), torch.zeros_like(acc)).to(torch.float32)
    return m if output_norm else torch.clamp(m, 0.0, 1.0)


def normalization_frame_sharded(frames_shard, nframes: int, normalize, ref_index: int = 0, lite: bool = False,
                                ctx=None, stats: Optional[Callable] = None, factors: Optional[Callable] = None,
                                group=None):
    """do_normalization for frame-sharded input.  Rank r holds
    frame_shards(N, world)[r] whole.  Returns (offset, mul, scale) of all N
    frames (numpy float64, identical on every rank) and raises
    NormalizationError for a failed frame, as the single-GPU path does.
    `stats(frames) -> NormStats` and `factors(normalize, NormStats, ref_index,
    lite) -> (off, mul, scale)` default to the HIP estimator kernels and the
    C-ABI factor arithmetic; tests inject CPU versions."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from . import normalization as Nz
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    shards = frame_shards(nframes, world)
    f0, f1 = shards[rank]
    if frames_shard.shape[0] != f1 - f0:
        raise ValueError(f"rank {rank} holds {frames_shard.shape[0]} frames, shard is {shards[rank]}")
    if int(normalize) == int(Nz.Normalization.NO_NORM):
        return np.zeros(nframes), np.ones(nframes), np.ones(nframes)
    st = stats(frames_shard) if stats is not None else Nz.norm_stats_device(ctx, frames_shard, lite)
    # one row per frame: median, mad, location, scale, ngood, status (exact in f64)
    nmax = max(b - a for a, b in shards)
    tab = torch.zeros((nmax, 6), dtype=torch.float64)
    k = f1 - f0
    tab[:k, :4] = torch.from_numpy(st.as_table())
    tab[:k, 4] = torch.from_numpy(np.asarray(st.ngood, np.float64))
    tab[:k, 5] = torch.from_numpy(np.asarray(st.status, np.float64))
    dev = frames_shard.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    tab = tab.to(dev)
    got = [torch.empty_like(tab) for _ in range(world)]
    dist.all_gather(got, tab, group=group)
    full = torch.cat([g[: b - a] for g, (a, b) in zip(got, shards)]).cpu().numpy()
    allst = Nz.NormStats(full[:, 0].copy(), full[:, 1].copy(), full[:, 2].copy(), full[:, 3].copy(),
                         full[:, 4].astype(np.int64), full[:, 5].astype(np.int32))
    fn = factors if factors is not None else (lambda nm, s, ri, li: Nz.factors(nm, s, ri, li))
    return fn(normalize, allst, ref_index, lite)


def _shard_args(args, f0: int, f1: int):
    """The per-frame arrays of StackingArgs restricted to frames [f0, f1)."""
    import dataclasses
    cut = lambda a: None if a is None else a[f0:f1]
    return dataclasses.replace(args, scale=cut(args.scale), offset=cut(args.offset), mul=cut(args.mul),
                               shiftx=cut(args.shiftx), weights=cut(args.weights))


def max_flagged(npix: int, world: int, nmax: int, byte_budget: int = 256 << 20) -> int:
    """Most order-sensitive pixels the frame-sharded mean recomputes from
    all-gathered columns: the gather holds world x nmax x k floats on every
    rank, bounded by `byte_budget` and by 1/16 of the image (beyond that the
    all-to-all transpose, (world - 1) / world of a shard per rank, moves less)."""
    return min(npix // 16, byte_budget // max(1, 4 * world * nmax))


def stack_frame_sharded(frames_shard, nframes: int, args, method: int = 0, ctx=None,
                        compute: Optional[Callable] = None, partial: Optional[Callable] = None,
                        finish: Optional[Callable] = None, group=None, post: Optional[Callable] = None,
                        columns: Optional[Callable] = None, pipeline: int = 4, ctxs=None):
    """Stack N frames sharded by frame over the ranks (rank r holds
    frame_shards(N, world)[r] whole, [n_r, H, W]).  Returns (full image
    [H, W] on every rank, (rejected_low, rejected_high) totals).

    NO_REJEC mean without weights: partial sums + counts, all-reduced (no
    transpose), with the exactness guard: pixels whose f64 sums are not
    provably order-independent are recomputed from their gathered columns in
    frame order.  Everything else: all-to-all to row bands, then the
    row-band stack (stack_distributed).  `partial(frames, args) -> (sum f64,
    count int32, amin f32, amax f32)`, `finish(sum, count, amin, amax) ->
    (image, flag)`, `columns(frames, args, idx) -> [n, k]` and `compute`
    default to the HIP kernels through `ctx`; tests inject CPU versions to
    check the decomposition with gloo.  `pipeline` > 1: the rejection path's
    transpose runs in that many row sub-chunks under the stack
    (stack_frame_sharded_pipelined; `ctxs`: extra Contexts its sub-chunk
    stacks alternate over); 0 or 1: one all-to-all of the whole band, then
    the stack."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    f0, f1 = frame_shards(nframes, world)[rank]
    _, H, W = frames_shard.shape
    mean_split = (method == 0 and int(args.type_of_rejection) == 0 and args.weights is None)

    def _rows():       # whole columns: the transpose to row bands, then the band stack
        if pipeline and pipeline > 1:
            return stack_frame_sharded_pipelined(frames_shard, nframes, args, method, ctx, compute, group, post,
                                                 subchunks=pipeline, ctxs=ctxs)
        band = transpose_frames_to_bands(frames_shard, nframes, group)
        return stack_distributed(band, H, args, method, ctx, compute, group, post)

    if mean_split:
        sargs = _shard_args(args, f0, f1)
        if partial is None:
            sum_, count, amin, amax = ctx.mean_partial_guard_device(frames_shard, sargs)
        else:
            sum_, count, amin, amax = partial(frames_shard, sargs)
        dist.all_reduce(sum_, group=group)
        dist.all_reduce(count, group=group)
        dist.all_reduce(amin, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(amax, op=dist.ReduceOp.MAX, group=group)
        if finish is None:
            full, flag = ctx.mean_finish_guard_device(sum_, count, amin, amax, output_norm=args.output_norm)
        else:
            full, flag = finish(sum_, count, amin, amax)
        # pixels whose f64 sums depend on the order (identical on every rank:
        # the reduced tables are): their columns are gathered and summed in
        # frame order, the order the single-device kernels restate
        idx = torch.nonzero(flag.reshape(-1)).reshape(-1)
        shards = frame_shards(nframes, world)
        nmax = max(b - a for a, b in shards)
        # the flagged columns are all-gathered whole ([world, nmax, k] floats
        # on every rank): past a budget the row-band path, exact by
        # construction, moves less (the flag is the same on every rank, so
        # every rank takes the same branch)
        if idx.numel() > max_flagged(H * W, world, nmax):
            return _rows()
        if idx.numel():
            cols = (ctx.gather_columns_device(frames_shard, sargs, idx) if columns is None
                    else columns(frames_shard, sargs, idx))
            pad = torch.zeros((nmax, idx.numel()), dtype=cols.dtype, device=cols.device)
            pad[: cols.shape[0]] = cols
            got = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(got, pad, group=group)
            allc = torch.cat([g[: b - a] for g, (a, b) in zip(got, shards)])
            full.view(-1)[idx] = _sequential_means(allc, bool(args.output_norm)).to(full.device)
        return _output_norm(full, args, ctx, post), (0, 0)
    return _rows()
