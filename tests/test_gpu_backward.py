"""Forward + loss + BACKWARD parity of the HIP path against the fp64 CPU oracle at the
benchmark and BASELINE.json config shapes (GPU).

* north star (BASELINE metric / configs[2]): FACT_CLIP, HAViD holdout dims, T=4096, the bench's
  two seg10 videos (seeds 1, 2) in one lockstep batch -- exactly the step bench.py times (split-K
  dW over 8192 stacked rows, 128x64 wide tiles, lockstep split nodes).  TDU segment counts equal
  the oracle's at these weights ([103, 27] and [89, 75]); batch loss within 1e-4 relative; every
  parameter gradient within 2e-3 (sampled entries, norm and sum).  The same batch run as two
  single-video steps gives the same mean gradient (the data-parallel equivalence on the real model:
  DP over whole videos averages exactly these per-video gradients).
* configs[1]: FACT_CLIP at HAViD dims with T=2048 (fp32; the bf16 perf mode reports its own S).
* configs[0]: vanilla FACT at Breakfast dims (MS-TCN++ 'm2' frame branch, hid/a/f dim 512,
  ntoken 60, C=48), T=512.
"""
import numpy as np
import pytest
import torch

from helpers import GruKinks, compare_grads, oracle_batch
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _gpu_step(net, vids, dp=None):
    """One forward + loss + backward.  dp (factmx.dp.DataParallel, world size 1): gradients land in
    its flat buffer exactly as in bench.py's timed step -- the MS-TCN backward then takes the deferred
    batched weight-gradient GEMMs (uniformly strided gradient views); without it every .grad is its
    own allocation and the per-layer interleaved GEMMs run."""
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    labs = [torch.from_numpy(l_).to(DEV) for _, l_ in vids]
    if dp is not None:
        dp.zero_grad()
    else:
        for p in net.parameters():
            p.grad = None
    loss, saves = net(seqs, labs, compute_loss=True)
    loss.backward()
    if dp is not None:
        dp.finish_gradients()
    torch.cuda.synchronize()
    return loss.item(), saves


def _segments(net):
    import bench
    return bench.video_segments(net)


def _video_records(net, nvid):
    """Per video, per block: (frame_clogit (T, C), tdu) of the last forward.  A lockstep batch keeps
    every video's views in blk._vrec; the per-video path leaves only the last video's attributes."""
    blocks = list(net.block_list)
    if all(getattr(b, "_vrec", None) is not None and len(b._vrec) == nvid for b in blocks):
        return [[(b._vrec[v]["frame_clogit"], b._vrec[v].get("tdu")) for b in blocks] for v in range(nvid)]
    return [None] * (nvid - 1) + [[(b.frame_clogit, getattr(b, "tdu", None)) for b in blocks]]


def _check_forward(net, spec, outs, saves, text):
    """Per-video predictions identical; for EVERY video of a lockstep batch (the last one on the
    per-video path) per-frame logits of every block within 1e-3 and TDU boundaries identical."""
    for v, out in enumerate(outs):
        pred = fo.predict(spec, out, None if text is None else text.double().cpu())
        np.testing.assert_array_equal(saves[v]["pred"], pred.numpy(), err_msg=f"video {v}")
    recs = _video_records(net, len(outs))
    assert recs[-1] is not None
    for v, (got, out) in enumerate(zip(recs, outs)):
        if got is None:
            continue
        for i, ((fcl, tdu), rec) in enumerate(zip(got, out["blocks"])):
            if rec["type"] == "U":
                np.testing.assert_array_equal(tdu.start32.cpu().numpy(), rec["tdu"].starts, err_msg=f"v{v} block {i}")
                np.testing.assert_array_equal(tdu.end32.cpu().numpy(), rec["tdu"].ends, err_msg=f"v{v} block {i}")
            err = (fcl[:, 0].double().cpu() - rec["frame_clogit"]).abs().max().item()
            assert err < 1e-3, f"video {v} block {i}: per-frame logits differ by {err}"


def test_north_star_lockstep_backward_vs_oracle(monkeypatch):
    import bench
    from factmx.models import blocks as blocks_mod
    cfg = bench.make_cfg()
    T, D, C = 4096, 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    assert blocks_mod._batchable(net, [torch.zeros(T, 1, device=DEV)] * 2)
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    S = _segments(net)
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    S_ref = [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs]
    assert S == S_ref, (S, S_ref)
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="lockstep T=4096: ")
    # data-parallel equivalence on the real model: the mean of the single-video gradients equals
    # the batch gradient (a GRU output at the ReLU kink may round to the other side between the
    # stacked and the single-video GEMMs: those blocks' GRU gradients are compared normwise)
    lock_gru = [(y, off) for y, off in kinks.gpu]
    acc = {n: torch.zeros_like(g) for n, g in grads.items()}
    for v in vids:
        _gpu_step(net, [v])
        for n, p in net.named_parameters():
            acc[n] += p.grad / len(vids)
    single = [y for y, _ in kinks.gpu[len(lock_gru):]]          # video-major, one per U block
    ublocks = [i for i, b in enumerate(net.block_list) if hasattr(b, "seg_update")]
    flips = set()
    for v in range(len(vids)):
        for j, (y, off) in enumerate(lock_gru):
            if ((y[off[v]:off[v + 1]] > 0) != (single[v * len(lock_gru) + j] > 0)).any():
                flips.add(f"block_list.{ublocks[j]}.seg_update.")
    for n, g in grads.items():
        if any(n.startswith(f) for f in flips):
            err = ((acc[n] - g).norm() / g.norm()).item()
            assert err <= 2e-2, (n, "normwise", err)
        else:
            err = (acc[n] - g).abs().max().item()
            assert err <= 1e-3 * g.abs().max().item() + 1e-7, (n, err)


def test_fact_clip_T2048_vs_oracle(monkeypatch):
    import bench
    cfg = bench.make_cfg()
    T, D, C = 2048, 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (3, 4)]
    kinks = GruKinks(monkeypatch)
    loss, saves = _gpu_step(net, vids)
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs]
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="T=2048: ")


def test_breakfast_vanilla_fact_vs_oracle(monkeypatch):
    import bench
    cfg = bench.make_cfg_breakfast()
    T, D, C = bench.BF_T, 2048, bench.BF_NCLS
    net, _ = bench.build_model(cfg, D, C, device=DEV, seed=0, clip=False)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    kinks = GruKinks(monkeypatch)
    loss, saves = _gpu_step(net, vids)
    spec = fo.resolve_spec(cfg, D, C, clip=False)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, None)
    _check_forward(net, spec, outs, saves, None)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="breakfast: ")


def test_ragged_lockstep_backward_vs_oracle(monkeypatch):
    """A ragged lockstep batch (T = 4096 and 2900, HAViD-holdout dims: the reference's DataLoader yields
    variable-length videos, dataset.py:106-131) against the fp64 oracle run per video: TDU segments and
    predictions identical, every video's per-frame logits within 1e-3, loss within 1e-4, gradients."""
    import bench
    from factmx.models import blocks as blocks_mod
    cfg = bench.make_cfg()
    D, C = 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for T, s in ((4096, 1), (2900, 5))]
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    assert blocks_mod._batchable(net, seqs)
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    assert net._vb.ragged and net._vb.Ts == [4096, 2900]
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="ragged: ")


def test_ntoken75_T4096_train_and_eval_vs_oracle(monkeypatch):
    """FACT.ntoken 75 (havid_view0_lh_pt_holdout.yaml:75) at T=4096: more than 64 action tokens take the
    fused decoder (token blocks of 64), the small-MHA / attention-over-T query blocks and the loss table
    on the lockstep path.  Train mode: loss, segments, logits and gradients vs the fp64 oracle; eval
    mode: the same forward (predictions, logits, segments) without a loss."""
    import bench
    cfg = bench.make_cfg(ntoken=75)
    T, D, C = 4096, 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="ntoken 75: ")
    net.eval()
    with torch.no_grad():
        saves = net([torch.from_numpy(f).to(DEV) for f, _ in vids], [torch.from_numpy(l_).to(DEV) for _, l_ in vids],
                    compute_loss=False)
    torch.cuda.synchronize()
    _check_forward(net, spec, outs, saves, text)


def test_shipped_yaml_training_step_full_shape():
    """The reference's havid_view0_lh_pt_holdout.yaml as shipped (Bi.dropout 0.2, FACT.cmr 0.3, time mask
    on, ntoken 75) at full shape on a ragged lockstep batch (T = 4096 + 2900): the training step runs the
    fused paths (lockstep, fused decoder with dropout at every site), its loss and every gradient are
    finite, and the same torch seed reproduces the step bit for bit (counter-based dropout masks, channel
    masking and time mask drawn from the seeded generators: torch's and Python's).  With dropout, cmr and the time mask off the
    same shape is held to the oracle by test_ntoken75_T4096_train_and_eval_vs_oracle / the ragged test."""
    import bench
    from factmx.models import blocks as blocks_mod
    cfg = bench.make_cfg_shipped()
    D, C = 2048, 75
    net, _ = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for T, s in ((4096, 1), (2900, 5))]
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    assert blocks_mod._batchable(net, seqs)

    def run():
        import random
        random.seed(123)            # the time mask draws its spans from Python's random (basic.py:35-47)
        np.random.seed(123)
        torch.manual_seed(123)
        torch.cuda.manual_seed(123)
        loss, saves = _gpu_step(net, vids)
        grads = [p.grad.detach().clone() for p in net.parameters()]
        return loss, grads, saves

    l1, g1, s1 = run()
    l2, g2, s2 = run()
    assert np.isfinite(l1), l1
    assert all(torch.isfinite(g).all() for g in g1)
    assert l1 == l2, (l1, l2)
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    for a, b in zip(s1, s2):
        np.testing.assert_array_equal(a["pred"], b["pred"])


@pytest.mark.parametrize("case", [((2, 1),), ((5, 2), (40, 5)), ((12, 3), (300, 10))],
                         ids=["T2", "T5+40", "T12+300"])
def test_short_videos_vs_oracle(case, monkeypatch):
    """Videos far shorter than the benchmark's (2 to 300 frames, one to ten ground-truth segments) at
    HAViD-holdout dims: MS-TCN dilations beyond the video length (zero padding only), one-segment TDU
    outputs, fewer keys than the fused attention cores' tiles, and a ragged lockstep batch whose videos
    differ 8x / 25x in length.  TDU segments and predictions identical to the fp64 oracle, per-frame
    logits within 1e-3, loss within 1e-4, every gradient.  (T=1 is left out: the reference's smoothing
    loss averages over the T-1 neighbouring-frame pairs and is NaN there, the oracle's likewise.)"""
    import bench
    cfg = bench.make_cfg()
    D, C = 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=7 + i, nseg=n) for i, (T, n) in enumerate(case)]
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what=f"short {case}: ")


@pytest.mark.parametrize("nvid", [16, 17])
def test_many_videos_vs_oracle(nvid, monkeypatch):
    """The widest lockstep batch (MAX_LOCKSTEP_VIDEOS = 16 ragged videos: every per-video offset table
    of the ragged convolutions, GRUs and fused attention cores full) and one video more (17: the
    batch leaves the lockstep path for the reference's one-video-at-a-time loop) at HAViD-holdout
    dims, lengths 33 to 609 frames, against the fp64 oracle: segments, predictions, per-frame logits
    of every video, the mean loss and every gradient."""
    import bench
    from factmx.models import blocks as blocks_mod
    cfg = bench.make_cfg()
    D, C = 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    Ts = [33 + (i * 233) % 589 for i in range(nvid)]
    vids = [bench.make_video(T, D, C, cfg, seed=20 + i, nseg=min(10, T // 8)) for i, T in enumerate(Ts)]
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    assert blocks_mod._batchable(net, seqs) == (nvid <= blocks_mod.MAX_LOCKSTEP_VIDEOS)
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    if nvid <= blocks_mod.MAX_LOCKSTEP_VIDEOS:
        assert net._vb.Ts == Ts
        S = _segments(net)
        assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what=f"{nvid} videos: ")


def test_holdout_labels_vs_oracle(monkeypatch):
    """Frames labelled with held-out classes (havid_view0_lh_pt_holdout.yaml's holdout_classes) at
    HAViD-holdout dims on a ragged lockstep batch: in video 0 one stretch of frames carries a held-out
    class (those frames leave the contrastive loss, blocks.py:728-744), video 1 is held out entirely
    (the unweighted FACT loss is returned, blocks.py:745-747).  Segments, predictions, logits, loss and every
    gradient against the fp64 oracle."""
    import bench
    cfg = bench.make_cfg()
    D, C = 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    (f0, l0), (f1, l1) = [bench.make_video(T, D, C, cfg, seed=s) for T, s in ((1024, 3), (700, 4))]
    l0 = l0.copy()
    l0[300:520] = bench.HOLDOUT[0]
    l1 = np.full_like(l1, bench.HOLDOUT[2])
    vids = [(f0, l0), (f1, l1)]
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="holdout: ")


def test_o2m_past_loss_table_limit_vs_oracle(monkeypatch):
    """One-to-many matching (loss.py:155-193) pairs EVERY ground-truth segment with a token, so a video
    with more than FX_LOSS_MAXK (512) segments overflows the fused loss-term table: the lockstep batch
    then computes its losses and predictions per video (the reference's MatchCriterion methods) on the
    lockstep outputs instead of failing.  Video 0 has 683 three-frame segments, video 1 is a seg10 video;
    segments, predictions, logits, loss and every gradient against the fp64 oracle."""
    import bench
    from factmx import native as nx
    from factmx.models import vloss
    cfg = bench.make_cfg()
    cfg.Loss.match = "o2m"
    D, C = 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    (f0, _), (f1, l1) = [bench.make_video(T, D, C, cfg, seed=s) for T, s in ((2048, 5), (1500, 6))]
    seen = [c for c in range(C) if c not in bench.HOLDOUT]
    l0 = np.asarray([seen[(i // 3) % 7] for i in range(2048)], dtype=np.int64)
    assert len(np.flatnonzero(np.diff(l0))) + 1 > nx.LOSS_MAXK
    vids = [(f0, l0), (f1, l1)]
    raised = []
    run = vloss.run

    def spy(*a, **k):
        try:
            return run(*a, **k)
        except vloss.TableTooLarge as e:
            raised.append(e.args[0])
            raise
    monkeypatch.setattr(vloss, "run", spy)
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    loss, saves = _gpu_step(net, vids, dp=DataParallel(net))
    assert raised == [[0]], raised
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    S = _segments(net)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="o2m > MAXK: ")
