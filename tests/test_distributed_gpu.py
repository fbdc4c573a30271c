"""The multi-GPU decomposition (siril_amd/distributed.py) over RCCL on the
box's one MI355X: a world-1 `nccl` process group, so every collective the
8-GPU path issues -- the frame-shard -> row-band `all_to_all_single` (16-bit
samples as float16 bits), the output `all_gather`, the rejection-count and
partial-sum `all_reduce`s (f64 sums, int32 counts, MIN / MAX bounds), the
flagged-column and normalization-table `all_gather`s -- runs through RCCL on
hardware, with the HIP kernels computing (no injected CPU compute).  The
results must equal the oracle's single-process stack of all frames
bit for bit (reference: row blocks median_and_mean.c:295-356; the
decomposition itself is checked at world 2 / 3 / 8 with gloo in
tests/test_distributed.py)."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    from siril_amd import distributed as D
    D.COLLECTIVE_AT_WORLD1 = True          # these tests exist to run the exchange through RCCL
    yield dist
    D.COLLECTIVE_AT_WORLD1 = False
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def ctx():
    from siril_amd import stacking
    c = stacking.Context(0)
    yield c
    c.close()


def _frames(n, h, w, seed):
    from siril_amd import synth
    fr = synth.frames_numpy(n, h, w, seed=seed)
    fr[3, 2, :] = 0.0                           # missing samples
    fr[:, 5, 7] = 0.0                           # an all-zero column
    return fr


def test_rccl_transpose_float_and_16bit(pg):
    """all_to_all_single of the frame shard into the row band (world 1: the
    whole frame stack), float32 and 16-bit (moved as float16 bits)."""
    import torch
    from siril_amd import distributed as D
    fr = _frames(9, 33, 70, seed=1)
    t = torch.from_numpy(fr).cuda()
    band = D.transpose_frames_to_bands(t, fr.shape[0])
    assert np.array_equal(band.cpu().numpy().view(np.uint32), fr.view(np.uint32))
    u = (fr * 60000).astype(np.uint16)
    b16 = D.transpose_frames_to_bands(torch.from_numpy(u.view(np.int16)).cuda(), fr.shape[0])
    assert b16.dtype == torch.int16
    assert np.array_equal(b16.cpu().numpy().view(np.uint16), u)


@pytest.mark.parametrize("pipeline", [0, 3])
@pytest.mark.parametrize("rtype,onorm", [(5, False), (2, False), (1, False), (5, True)])
def test_rccl_frame_sharded_rejection(pg, ctx, oracle, rtype, onorm, pipeline):
    """Rejection stacks of frame-sharded input: all-to-all to row bands,
    the HIP row-band stack, all_gather of the output, all_reduce of the
    rejection totals; -output_norm rescales the gathered image.  pipeline 3:
    the band in three row sub-chunks, each exchanged from a side stream by an
    asynchronous RCCL all_to_all_single while the previous one stacks."""
    import torch
    from oracle import headless_ref as HR
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    fr = _frames(37, 24, 96, seed=10 + rtype)
    if onorm:
        fr[:, 8, :] *= 1.8
    full, rej = D.stack_frame_sharded(torch.from_numpy(fr).cuda(), fr.shape[0],
                                      StackingArgs(Rejection(rtype), (3.0, 3.0), output_norm=onorm), 0, ctx=ctx,
                                      pipeline=pipeline)
    out, rl, rh, counts = oracle.stack_rows(fr, rtype, (3.0, 3.0), nthreads=2, output_norm=onorm)
    if onorm:
        out = HR.norm_to_0_1_range(out)
    assert np.array_equal(full.cpu().numpy().view(np.uint32), out.view(np.uint32))
    assert rej == (int(counts[0]), int(counts[1]))


def test_rccl_pipelined_two_contexts(pg, ctx, oracle):
    """The pipelined transpose with the sub-chunk stacks alternating over two
    Contexts on two streams (one launch's tail under the next one's start):
    same image and totals as the oracle."""
    import torch
    from siril_amd import distributed as D, stacking as S
    from siril_amd.stacking import Rejection, StackingArgs
    fr = _frames(41, 30, 96, seed=21)
    ctx2 = S.Context(0)
    try:
        for rt in (5, 2):
            full, rej = D.stack_frame_sharded_pipelined(torch.from_numpy(fr).cuda(), fr.shape[0],
                                                        StackingArgs(Rejection(rt), (3.0, 3.0)), 0, subchunks=5,
                                                        ctxs=[ctx, ctx2])
            out, rl, rh, counts = oracle.stack_rows(fr, rt, (3.0, 3.0), nthreads=2)
            assert np.array_equal(full.cpu().numpy().view(np.uint32), out.view(np.uint32)), rt
            assert rej == (int(counts[0]), int(counts[1])), rt
    finally:
        ctx2.close()


def test_rccl_frame_sharded_16bit(pg, ctx, oracle):
    """16-bit frame shards: the transpose moves them as float16 bits, the
    16-bit HIP stack (float output) equals apply_rejection_ushort's."""
    import torch
    from siril_amd import distributed as D
    from siril_amd.stacking import Rejection, StackingArgs
    u = (_frames(40, 20, 64, seed=7) * 60000).astype(np.uint16)
    out, rl, rh, counts = oracle.stack_rows_u16(u, 5, (3.0, 3.0), nthreads=2, use_32bit_output=True)
    for pipeline in (0, 4):
        full, rej = D.stack_frame_sharded(torch.from_numpy(u.view(np.int16)).cuda(), u.shape[0],
                                          StackingArgs(Rejection.WINSORIZED, (3.0, 3.0)), 0, ctx=ctx,
                                          pipeline=pipeline)
        assert np.array_equal(full.cpu().numpy().view(np.uint32), np.asarray(out, np.float32).view(np.uint32))
        assert rej == (int(counts[0]), int(counts[1]))


@pytest.mark.parametrize("norm", [3, 4])
def test_rccl_frame_sharded_mean_partial_sums(pg, ctx, oracle, norm):
    """NO_REJEC mean without weights: HIP partial sums all-reduced over RCCL
    (f64 sums, counts, MIN / MAX), the exactness guard, and the flagged
    columns (~1e-9 next to ~1 samples) all-gathered and summed in frame
    order; equal to the oracle's mean of all frames."""
    import torch
    from oracle import headless_ref as HR
    from siril_amd import distributed as D
    from siril_amd.stacking import Normalization, Rejection, StackingArgs
    n = 13
    fr = _frames(n, 16, 40, seed=19)
    rng = np.random.default_rng(norm)
    scale = 1.0 + 0.05 * rng.standard_normal(n)
    offset = 0.055 + 0.002 * rng.standard_normal(n)
    mul = 1.0 + 0.05 * rng.standard_normal(n)
    even = (np.arange(n) % 2 == 0)[:, None]
    tiny = ((offset / scale).astype(np.float32)[:, None] if norm in (1, 3)
            else np.full((n, 1), 3e-9, np.float32))
    fr[:, 3, 2:8] = np.where(even, tiny, np.float32(0.9))
    args = StackingArgs(Rejection(0), (3.0, 3.0), Normalization(norm), scale=scale, offset=offset, mul=mul,
                        output_norm=True)
    full, rej = D.stack_frame_sharded(torch.from_numpy(fr).cuda(), n, args, 0, ctx=ctx)
    out, rl, rh, counts = oracle.stack_rows(fr, 0, (3.0, 3.0), nthreads=2, output_norm=True, norm=norm,
                                            scale=scale, offset=offset, mul=mul)
    out = HR.norm_to_0_1_range(out)
    assert np.array_equal(full.cpu().numpy().view(np.uint32), out.view(np.uint32))
    assert rej == (0, 0)


@pytest.mark.parametrize("normalize,ref", [(3, 0), (4, 5), (1, 2)])
def test_rccl_frame_sharded_normalization(pg, ctx, normalize, ref):
    """The frame-sharded normalization: HIP estimators of the shard, the
    per-frame table all-gathered over RCCL (f64), the factor arithmetic;
    equal to the single-device pass over all frames."""
    import torch
    from siril_amd import distributed as D, normalization as Nz, synth
    from siril_amd.stacking import Normalization
    fr = synth.frames_numpy(11, 48, 58, seed=4)
    fr *= (1.0 + 0.05 * np.arange(11, dtype=np.float32))[:, None, None]
    fr += (0.01 * np.arange(11, dtype=np.float32))[:, None, None]
    t = torch.from_numpy(fr).cuda()
    got = D.normalization_frame_sharded(t, fr.shape[0], Normalization(normalize), ref, ctx=ctx)
    want = Nz.factors(Normalization(normalize), Nz.norm_stats_device(ctx, t), ref)
    for a, b in zip(got, want):
        assert np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))
