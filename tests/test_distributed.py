"""Row-band multi-process decomposition (siril_amd/distributed.py) with the
gloo backend on CPU, world size 2, 3 and 8 (the target node's rank count): the gathered image and the reduced
rejection totals must equal a single-process stack of the whole image.  The
per-band compute is the oracle here (CPU); on GPUs it is the HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_compute(frames_band, args, method):
    from oracle import oracle as O
    kw = {} if int(args.normalize) == 0 else dict(norm=int(args.normalize), scale=args.scale, offset=args.offset,
                                                    mul=args.mul)
    out, rl, rh, counts = O.stack_rows(frames_band.numpy(), int(args.type_of_rejection), args.sig,
                                       method=method, nthreads=1, output_norm=bool(args.output_norm), **kw)
    return torch.from_numpy(out), torch.tensor([int(counts[0]), int(counts[1])], dtype=torch.int64)


def _worker(rank, world, port, frames, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    y0, y1 = D.row_bands(frames.shape[1], world)[rank]
    band = torch.from_numpy(np.ascontiguousarray(frames[:, y0:y1]))
    full, rej = D.stack_distributed(band, frames.shape[1], StackingArgs(Rejection.WINSORIZED, (3.0, 3.0)),
                                    0, compute=_oracle_compute)
    if rank == 0:
        q.put((full.numpy(), rej))
    dist.barrier()
    dist.destroy_process_group()


def test_row_bands():
    from siril_amd.distributed import row_bands
    assert row_bands(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert row_bands(4000, 8)[-1] == (3500, 4000)
    for h, w in [(1, 1), (7, 8), (4000, 3)]:
        b = row_bands(h, w)
        assert b[0][0] == 0 and b[-1][1] == h and all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_row_band_stack(oracle, world):
    from siril_amd import synth
    frames = synth.frames_numpy(20, 11, 16, seed=3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, rej = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out, rl, rh, counts = oracle.stack_rows(frames, oracle.WINSORIZED, (3.0, 3.0), nthreads=2)
    assert np.array_equal(full.view(np.uint32), out.view(np.uint32))
    assert rej == (int(counts[0]), int(counts[1]))


def _np_norm(a, args):
    """The stack's per-sample normalization (gather_sample, median_and_mean.c
    :1644-1686) in numpy: f64 affine of the non-null samples, rounded to f32."""
    if int(args.normalize) == 0:
        return a
    out = np.empty_like(a)
    for f in range(a.shape[0]):
        x = a[f].astype(np.float64)
        if int(args.normalize) in (1, 3):
            y = (x * args.scale[f] - args.offset[f]).astype(np.float32)
            out[f] = np.where(a[f] != 0, y, np.float32(0))
        else:
            out[f] = ((x * args.scale[f]) * args.mul[f]).astype(np.float32)
    return out


def _np_partial(frames_shard, args):
    """CPU stand-in for sgpu_mean_partial_guard_device (test infrastructure):
    f64 sum and count of the non-zero normalized samples in frame order, and
    their smallest / largest magnitude."""
    a = _np_norm(frames_shard.numpy(), args)
    s = np.zeros(a.shape[1:], np.float64)
    k = np.zeros(a.shape[1:], np.int32)
    lo = np.full(a.shape[1:], np.inf, np.float32)
    hi = np.zeros(a.shape[1:], np.float32)
    for f in range(a.shape[0]):
        nz = a[f] != 0
        s[nz] += a[f][nz].astype(np.float64)
        k += nz
        lo[nz] = np.minimum(lo[nz], np.abs(a[f][nz]))
        hi[nz] = np.maximum(hi[nz], np.abs(a[f][nz]))
    return torch.from_numpy(s), torch.from_numpy(k), torch.from_numpy(lo), torch.from_numpy(hi)


def _np_finish(s, k, lo, hi, output_norm=False):
    from siril_amd import distributed as D
    flag = (~D.partial_sums_exact(k, lo, hi)).to(torch.uint8)
    s, k = s.numpy(), k.numpy()
    with np.errstate(invalid="ignore", divide="ignore"):
        m = np.where(k > 0, s / np.maximum(k, 1), 0.0).astype(np.float32)
    return torch.from_numpy(m if output_norm else np.clip(m, 0, 1).astype(np.float32)), flag


def _np_columns(frames_shard, args, idx):
    a = _np_norm(frames_shard.numpy(), args)
    return torch.from_numpy(np.ascontiguousarray(a.reshape(a.shape[0], -1)[:, idx.numpy()]))


def _np_post(full):
    """CPU stand-in for sgpu_norm_to_0_1_range_device (test infrastructure)."""
    from oracle import headless_ref as HR
    return torch.from_numpy(HR.norm_to_0_1_range(full.numpy()))


def _sharded_worker(rank, world, port, frames, rtype, q, onorm=False, norm=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    n = frames.shape[0]
    f0, f1 = D.frame_shards(n, world)[rank]
    shard = torch.from_numpy(np.ascontiguousarray(frames[f0:f1]))
    # the all-to-all itself, 16-bit samples included (moved as float16 bits)
    y0, y1 = D.row_bands(frames.shape[1], world)[rank]
    ok_t = True
    for mode in ("all_to_all", "p2p"):
        band = D.transpose_frames_to_bands(shard, n, mode=mode)
        ok_t = ok_t and np.array_equal(band.numpy().view(np.uint32), frames[:, y0:y1].view(np.uint32))
        s16 = torch.from_numpy((frames[f0:f1] * 30000).astype(np.int16))
        b16 = D.transpose_frames_to_bands(s16, n, mode=mode)
        ok_t = ok_t and np.array_equal(b16.numpy(), (frames[:, y0:y1] * 30000).astype(np.int16))
    if norm is None:
        args = StackingArgs(Rejection(rtype), (3.0, 3.0), output_norm=onorm)
    else:
        from siril_amd.stacking import Normalization
        args = StackingArgs(Rejection(rtype), (3.0, 3.0), Normalization(norm[0]), scale=norm[1], offset=norm[2],
                            mul=norm[3], output_norm=onorm)
    full, rej = D.stack_frame_sharded(shard, n, args, 0, compute=_oracle_compute, partial=_np_partial,
                                      finish=lambda a, b, c, d: _np_finish(a, b, c, d, onorm), post=_np_post,
                                      columns=_np_columns)
    if rank == 0:
        q.put((full.numpy(), rej, ok_t))
    else:
        q.put((None, None, ok_t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rtype,onorm", [(2, 0, False), (3, 0, False), (2, 5, False), (3, 5, False),
                                               (2, 0, True), (3, 5, True), (8, 0, False), (8, 5, True)])
def test_gloo_frame_sharded_stack(oracle, world, rtype, onorm):
    """Frame-sharded input: NO_REJEC mean through the partial-sum / count
    all-reduce, WINSORIZED through the all-to-all transpose to row bands;
    both equal the single-process oracle stack of all frames.  With
    -output_norm the unclamped result gets norm_to_0_1_range over the whole
    gathered image (median_and_mean.c:1774-1775), not per band."""
    from oracle import headless_ref as HR
    from siril_amd import synth
    frames = synth.frames_numpy(13, 10, 17, seed=9)
    frames[4, 2, :] = 0.0                       # missing samples
    frames[:, 7, 3] = 0.0                       # an all-zero column
    if onorm:
        frames[:, 8, :] *= 1.8                  # results above 1 (unclamped before the post-pass)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, frames, rtype, q, onorm))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(g[2] for g in got), "all-to-all transpose"
    full, rej = next((g[0], g[1]) for g in got if g[0] is not None)
    out, rl, rh, counts = oracle.stack_rows(frames, rtype, (3.0, 3.0), nthreads=2, output_norm=onorm)
    if onorm:
        out = HR.norm_to_0_1_range(out)
    assert np.array_equal(full.view(np.uint32), out.view(np.uint32))
    assert rej == (int(counts[0]), int(counts[1]))


@pytest.mark.parametrize("world,rtype,norm", [(2, 0, 3), (3, 0, 3), (3, 0, 4), (2, 5, 3), (3, 5, 1), (8, 0, 3)])
def test_gloo_frame_sharded_stack_normalized(oracle, world, rtype, norm):
    """Frame-sharded stack of normalized data whose additive offsets push
    samples below zero and next to it, plus columns mixing ~1e-9 and ~1
    samples (f64 partial sums NOT exact): the partial-sum guard flags those
    pixels and they are recomputed from their gathered columns in frame
    order; every pixel equals the single-process oracle stack."""
    from siril_amd import distributed as D, synth
    n = 13
    frames = synth.frames_numpy(n, 10, 17, seed=19)
    frames[5, 6, :] = 0.0
    rng = np.random.default_rng(norm)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.055 + 0.002 * rng.standard_normal(n)          # most samples -> around and below 0
    mul = 1.0 + 0.05 * rng.standard_normal(n)
    # columns whose normalized samples span ~2^30: even frames land within
    # rounding of zero (additive: x = offset / scale; multiplicative: x tiny)
    even = (np.arange(n) % 2 == 0)[:, None]
    tiny = ((offset / scale).astype(np.float32)[:, None] if norm in (1, 3)
            else np.full((n, 1), 3e-9, np.float32))
    frames[:, 3, 2:8] = np.where(even, tiny, np.float32(0.9))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, frames, rtype, q, True,
                                                       (norm, scale, offset, mul)))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, rej = next((g[0], g[1]) for g in got if g[0] is not None)
    from oracle import headless_ref as HR
    out, rl, rh, counts = oracle.stack_rows(frames, rtype, (3.0, 3.0), nthreads=2, output_norm=True, norm=norm,
                                            scale=scale, offset=offset, mul=mul)
    out = HR.norm_to_0_1_range(out)
    assert np.array_equal(full.view(np.uint32), out.view(np.uint32))
    assert rej == (int(counts[0]), int(counts[1]))
    if rtype == 0:
        a = _np_norm(frames, type("A", (), {"normalize": norm, "scale": scale, "offset": offset, "mul": mul})())
        _, k, lo, hi = _np_partial(torch.from_numpy(frames), type("A", (), {"normalize": 0})())
        lo = torch.from_numpy(np.where(a != 0, np.abs(a), np.inf).min(0).astype(np.float32))
        hi = torch.from_numpy(np.abs(a).max(0).astype(np.float32))
        k = torch.from_numpy((a != 0).sum(0).astype(np.int32))
        assert int((~D.partial_sums_exact(k, lo, hi)).sum()) >= 4       # the guard fired


def _oracle_norm_stats(frames):
    """CPU stand-in for the HIP estimator kernels (test infrastructure)."""
    from oracle import oracle as O
    from siril_amd.normalization import NormStats
    rows = [O.norm_stats(f) for f in np.asarray(frames)]
    col = lambda i, t: np.array([r[i] for r in rows], t)
    return NormStats(col(1, np.float64), col(2, np.float64), col(3, np.float64), col(4, np.float64),
                     col(5, np.int64), col(0, np.int32))


def _norm_worker(rank, world, port, frames, normalize, ref, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    n = frames.shape[0]
    f0, f1 = D.frame_shards(n, world)[rank]
    shard = torch.from_numpy(np.ascontiguousarray(frames[f0:f1]))
    q.put((rank, D.normalization_frame_sharded(shard, n, normalize, ref, stats=_oracle_norm_stats)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,normalize,ref", [(2, 3, 0), (3, 3, 5), (3, 1, 2), (2, 4, 7), (3, 2, 0), (8, 3, 9)])
def test_gloo_frame_sharded_normalization(oracle, world, normalize, ref):
    """Normalization of frame-sharded input: per-rank estimators of whole
    frames + an all-gather of the per-frame tables give, on every rank,
    exactly the factors of the single-process pass over all frames
    (normalization.c:150-185, 249-294), for every -norm= kind and a
    reference frame on any rank."""
    from siril_amd import normalization as Nz, synth
    from siril_amd.stacking import Normalization
    frames = synth.frames_numpy(11, 24, 29, seed=4)
    frames *= (1.0 + 0.05 * np.arange(11, dtype=np.float32))[:, None, None]
    frames += (0.01 * np.arange(11, dtype=np.float32))[:, None, None]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_norm_worker, args=(r, world, port, frames, normalize, ref, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = Nz.factors(Normalization(normalize), _oracle_norm_stats(frames), ref)
    for _, fac in got:
        for a, b in zip(fac, want):
            assert np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


def _transpose_worker(rank, world, port, frames, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    n, H = frames.shape[:2]
    f0, f1 = D.frame_shards(n, world)[rank]
    y0, y1 = D.row_bands(H, world)[rank]
    band = D.transpose_frames_to_bands(torch.from_numpy(np.ascontiguousarray(frames[f0:f1])), n)
    ok = tuple(band.shape) == (n, y1 - y0, frames.shape[2])
    ok = ok and np.array_equal(band.numpy().view(np.uint32), frames[:, y0:y1].view(np.uint32))
    try:                                           # p2p refuses layouts with idle ranks
        D.transpose_frames_to_bands(torch.from_numpy(np.ascontiguousarray(frames[f0:f1])), n, mode="p2p")
        ok = False
    except ValueError:
        pass
    q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n,h", [(5, 13), (13, 5), (3, 3)], ids=["empty-shards", "empty-bands", "both"])
def test_gloo_transpose_ragged_world8(n, h):
    """The all-to-all transpose at world 8 with ranks that hold no frame
    (nframes < world) and ranks whose row band is empty (H < world): every
    rank joins the one collective with zero-sized pieces (no rank
    may skip the exchange); the p2p mode refuses such layouts."""
    world = 8
    frames = np.random.default_rng(n * h).random((n, h, 6)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_transpose_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got)


def _flagged_worker(rank, world, port, frames, norm, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    from siril_amd.stacking import Normalization, Rejection, StackingArgs
    n = frames.shape[0]
    f0, f1 = D.frame_shards(n, world)[rank]
    shard = torch.from_numpy(np.ascontiguousarray(frames[f0:f1]))
    args = StackingArgs(Rejection(0), (3.0, 3.0), Normalization(norm[0]), scale=norm[1], offset=norm[2],
                        mul=norm[3], output_norm=True)
    used = {"cols": 0}

    def cols(fs, a, idx):
        used["cols"] += 1
        return _np_columns(fs, a, idx)
    full, _ = D.stack_frame_sharded(shard, n, args, 0, compute=_oracle_compute, partial=_np_partial,
                                    finish=lambda a, b, c, d: _np_finish(a, b, c, d, True), post=_np_post,
                                    columns=cols)
    q.put((rank, full.numpy() if rank == 0 else None, used["cols"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_frame_sharded_mean_most_flagged(oracle, world):
    """normalized data where the partial-sum guard flags most of
    the image (every column mixes samples next to zero with ~1): past
    max_flagged the stack takes the all-to-all + row-band path instead of
    all-gathering the flagged columns (no column gather on any rank), and
    still equals the single-process oracle stack bit for bit."""
    from oracle import headless_ref as HR
    from siril_amd import distributed as D, synth
    n, H, W = 13, 10, 17
    frames = synth.frames_numpy(n, H, W, seed=29)
    rng = np.random.default_rng(5)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.055 + 0.002 * rng.standard_normal(n)
    mul = np.ones(n)
    even = (np.arange(n) % 2 == 0)[:, None, None]
    frames = np.where(even, (offset / scale).astype(np.float32)[:, None, None], np.float32(0.9)) \
        + np.float32(1e-9) * frames
    frames = frames.astype(np.float32)
    nmax = max(b - a for a, b in D.frame_shards(n, world))
    assert D.max_flagged(H * W, world, nmax) < H * W // 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flagged_worker, args=(r, world, port, frames, (3, scale, offset, mul), q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(g[2] == 0 for g in got), "flagged columns were gathered past the budget"
    full = next(g[1] for g in got if g[1] is not None)
    out = oracle.stack_rows(frames, 0, (3.0, 3.0), nthreads=2, output_norm=True, norm=3, scale=scale,
                            offset=offset, mul=mul)[0]
    out = HR.norm_to_0_1_range(out)
    assert np.array_equal(full.view(np.uint32), out.view(np.uint32))


def _pipe_worker(rank, world, port, frames, rtype, ks, q, u16=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    n = frames.shape[0]
    f0, f1 = D.frame_shards(n, world)[rank]
    shard = torch.from_numpy(np.ascontiguousarray(frames[f0:f1]))
    args = StackingArgs(Rejection(rtype), (3.0, 3.0))
    res = []
    seen = []

    def compute(band, a, method):
        seen.append(tuple(band.shape))
        b = band.numpy()
        if u16:             # the 16-bit band arrives as int16 bits: check it, stack its float image
            b = b.view(np.uint16).astype(np.float32) / np.float32(65535.0)
        return _oracle_compute(torch.from_numpy(np.ascontiguousarray(b)), a, method)

    src = shard
    if u16:
        src = torch.from_numpy((frames[f0:f1] * 65535).astype(np.uint16).view(np.int16))
    for k in ks:
        seen.clear()
        full, rej = D.stack_frame_sharded_pipelined(src, n, args, 0, compute=compute, subchunks=k)
        res.append((k, full.numpy() if rank == 0 else None, rej, list(seen)))
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,h,rtype,u16", [(2, 13, 10, 5, False), (3, 13, 11, 2, False),
                                                 (8, 17, 21, 5, False), (8, 5, 13, 5, False),
                                                 (3, 14, 9, 5, True)],
                         ids=["w2", "w3-sigma", "w8", "w8-empty-shards", "w3-16bit"])
def test_gloo_pipelined_transpose_stack(oracle, world, n, h, rtype, u16):
    """The pipelined frame-shard -> row-band path: the band cut
    into K row sub-chunks, each one staged, exchanged with one asynchronous
    all_to_all_single and stacked while the next one moves.  For K = 1, 2,
    3 and K larger than the band (empty sub-chunks), with ranks holding no
    frame (n < world), the image and the rejection totals equal the
    single-process oracle stack of all frames bit for bit, and every
    sub-chunk reaches the stack as a whole-column [n, rows, W] block."""
    from siril_amd import distributed as D, synth
    frames = synth.frames_numpy(n, h, 19, seed=31 + world)
    frames[1, 2, :] = 0.0
    if u16:
        frames = (np.round(frames * 65535) / 65535).astype(np.float32)
    ks = [1, 2, 3, h + 2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, frames, rtype, ks, q, u16))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src = frames
    if u16:
        src = ((frames * 65535).astype(np.uint16).astype(np.float32) / np.float32(65535.0)).astype(np.float32)
    out, rl, rh, counts = oracle.stack_rows(src, rtype, (3.0, 3.0), nthreads=2)
    bands = D.row_bands(h, world)
    for rank, res in got.items():
        for k, full, rej, seen in res:
            assert rej == (int(counts[0]), int(counts[1])), (rank, k)
            if full is not None:
                assert np.array_equal(full.view(np.uint32), out.view(np.uint32)), k
            split = D.sub_bands_lead if k > 1 else D.sub_bands      # the default lead-half split
            subs = [b1 - b0 for b0, b1 in split(bands[rank], k) if b1 > b0]
            assert seen == [(n, r, 19) for r in subs], (rank, k, seen)


def test_sub_bands():
    from siril_amd.distributed import sub_bands, sub_bands_lead
    assert sub_bands_lead((0, 500), 5) == [(0, 56), (56, 167), (167, 278), (278, 389), (389, 500)]
    for band, k in (((3, 3), 2), ((0, 3), 5), ((7, 108), 4), ((0, 1), 1)):
        sb = sub_bands_lead(band, k)
        assert len(sb) == k and sb[0][0] == band[0] and sb[-1][1] == band[1]
        assert all(sb[i][1] == sb[i + 1][0] and sb[i][0] <= sb[i][1] for i in range(k - 1))
    assert sub_bands((10, 20), 3) == [(10, 14), (14, 17), (17, 20)]
    assert sub_bands((5, 7), 4) == [(5, 6), (6, 7), (7, 7), (7, 7)]
    assert sub_bands((3, 3), 2) == [(3, 3), (3, 3)]


def _cap_worker(rank, world, port, frames, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    D.MAX_PIECE_BYTES = 4 * 19 * 3            # three rows of one frame: forces many sub-chunks
    n, H = frames.shape[:2]
    f0, f1 = D.frame_shards(n, world)[rank]
    y0, y1 = D.row_bands(H, world)[rank]
    shard = torch.from_numpy(np.ascontiguousarray(frames[f0:f1]))
    band = D.transpose_frames_to_bands(shard, n)
    ok = np.array_equal(band.numpy().view(np.uint32), frames[:, y0:y1].view(np.uint32))
    seen = []

    def compute(b, a, m):
        seen.append(tuple(b.shape))
        return _oracle_compute(b, a, m)
    full, rej = D.stack_frame_sharded_pipelined(shard, n, StackingArgs(Rejection.WINSORIZED, (3.0, 3.0)), 0,
                                                compute=compute, subchunks=2)
    q.put((rank, ok, full.numpy(), rej, seen))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_transpose_piece_cap():
    """Collectives past MAX_PIECE_BYTES are cut into row sub-chunks (RCCL's
    all_to_all_single corrupted 4 GiB pieces on the MI355X box,
    profiles/r06b_fs_check.log): with the cap lowered to a few rows, the plain
    transpose and the pipelined stack still deliver every band exactly, and
    the pipeline runs more sub-chunks than asked for."""
    from oracle import oracle as O
    from siril_amd import synth
    world = 3
    frames = synth.frames_numpy(11, 17, 19, seed=12)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cap_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out, rl, rh, counts = O.stack_rows(frames, O.WINSORIZED, (3.0, 3.0), nthreads=2)
    for rank, ok, full, rej, seen in got:
        assert ok, rank
        assert np.array_equal(full.view(np.uint32), out.view(np.uint32))
        assert rej == (int(counts[0]), int(counts[1]))
        assert len(seen) > 2 and all(r <= 1 for _, r, _ in seen), seen
