"""Data parallelism on the real kernels: a 2-rank step equals the 1-process
step on the concatenated batch.

Two ranks run as child processes on the box's single GPU with the gloo
backend (device tensors staged through host memory by ainp.dist.Comm); the
exchange points are the production ones:
  * CNNBLSTM: SyncBN forward/backward sums, SUM-all-reduced gradients
    (overlapped buckets), Adam;
  * GAN: SyncBN of G's 13 BatchNorms, D gradients averaged, the VGG target's
    batch max MAX-all-reduced, the hole/valid L1 sums SUM-all-reduced, the
    logged per-rank means averaged.
The reference is computed in this process on the whole batch.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(mode, tmp_path, world=2, timeout=240):
    port = _free_port()
    out = str(tmp_path / mode)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), mode,
                                       out], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    return [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.timeout(300)
def test_cnnblstm_dp2_equals_single_process(tmp_path):
    import dp_worker
    ref = dp_worker.run_cnnblstm()
    ranks = _run_ranks("cnnblstm", tmp_path)
    assert _rel(ranks[0]["loss"], ref["loss"]) < 1e-6
    # conv biases that feed a BatchNorm have an analytically zero gradient
    # (SURVEY Q10): their fp32 gradients are rounding noise, which Adam scales
    # to +-lr, so they are checked absolutely (lr = 1e-3)
    _check_state(ranks, ref)
    # the layer-0 input weights' gradients went to the reducer in 4 gate chunks
    # per direction, all-reduced as they completed
    assert ranks[0]["early_chunks"] == 8
    # the other side-stream weight gradients (encoder and decoder convs,
    # projection, BLSTM W_hh / biases / upper W_ih) were all-reduced from the
    # side stream as they were written -- the single-GPU overlaps kept under DP
    assert ranks[0]["side_reductions"] > 0
    assert ranks[0]["bad_storage"] == [] and ranks[1]["bad_storage"] == []


@pytest.mark.timeout(300)
def test_cnnblstm_dp2_device_collectives_keep_reduced_storage(tmp_path):
    """Gradients handed to gloo's async CUDA collectives (no host staging):
    the Work objects hold the reduced tensors until wait(), as RCCL's do, so a
    gradient autograd received by reference would be cloned on the compute
    stream before the side stream wrote it.  Every reduced buffer must be the
    storage of p.grad, and the result equal the host-staged run bit for bit."""
    dev = _run_ranks("cnnblstm:dev", tmp_path)
    host = _run_ranks("cnnblstm", tmp_path)
    for r in range(2):
        assert dev[r]["bad_storage"] == [], dev[r]["bad_storage"]
    assert dev[0]["side_reductions"] > 0 and dev[0]["early_chunks"] == 8
    assert torch.equal(dev[0]["loss"], host[0]["loss"])
    for k, v in host[0]["state"].items():
        assert torch.equal(dev[0]["state"][k], v), k
        assert torch.equal(dev[1]["state"][k], v), k


@pytest.mark.timeout(300)
def test_cnnblstm_dp2_fused_layer0_pair(tmp_path):
    """H = 64 (4H = 256 gate rows): each rank runs the fp32 layer-0 backward
    as the same single gemm_x6r launch as one GPU does and hands both
    directions' W_ih gradients to the reducer right behind it (no chunked
    side-stream GEMMs).  Matches the 1-process step on the whole batch, is
    bit-identical with and without the other side-stream hand-offs, and keeps
    the reduced buffers as the .grad storage under device collectives."""
    import dp_worker
    ref = dp_worker.run_cnnblstm(pair=True)
    on = _run_ranks("cnnblstm_pair:dev", tmp_path)
    off = _run_ranks("cnnblstm_pair_nodefer", tmp_path)
    for res in (on, off):
        assert res[0]["pair_reductions"] == 2 and res[0]["early_chunks"] == 0
        assert res[0]["bad_storage"] == [] and res[1]["bad_storage"] == []
    assert _rel(on[0]["loss"], ref["loss"]) < 1e-6
    _check_state(on, ref)
    assert torch.equal(on[0]["loss"], off[0]["loss"])
    for k, v in off[0]["state"].items():
        assert torch.equal(on[0]["state"][k], v), k
        assert torch.equal(on[1]["state"][k], v), k


@pytest.mark.timeout(300)
def test_cnnblstm_dp2_side_stream_reductions_bit_identical(tmp_path):
    """Under DP, the deferred / side-stream weight gradients are handed to the
    reducer from the side stream (no compute-stream join); the result is bit
    for bit the one with every weight gradient synchronous (deferral off)."""
    on = _run_ranks("cnnblstm", tmp_path)
    off = _run_ranks("cnnblstm_nodefer", tmp_path)
    assert off[0]["side_reductions"] == 0 < on[0]["side_reductions"]
    assert torch.equal(on[0]["loss"], off[0]["loss"])
    for k, v in off[0]["state"].items():
        assert torch.equal(on[0]["state"][k], v), k
        assert torch.equal(on[1]["state"][k], v), k


def _check_state(ranks, ref, tol=1e-5):
    bn_fed = {"encoder.0.bias", "encoder.3.bias", "encoder.6.bias", "decoder.0.bias",
              "decoder.3.bias"}
    for k, v in ref["state"].items():
        if k.endswith("num_batches_tracked"):
            assert torch.equal(ranks[0]["state"][k], v)
            continue
        if k in bn_fed:
            assert float((ranks[0]["state"][k] - v).abs().max()) <= 2.5e-3 * 2, k
        elif k.endswith("running_mean"):   # carries momentum x the BN-fed biases' noise
            assert float((ranks[0]["state"][k] - v).abs().max()) <= \
                5e-4 + tol * float(v.abs().max()), k
        else:
            assert _rel(ranks[0]["state"][k], v) < tol, k
        assert torch.equal(ranks[0]["state"][k], ranks[1]["state"][k]), k


@pytest.mark.timeout(300)
def test_cnnblstm_dp2_uneven_shards_equal_single_process(tmp_path):
    """Rank 0 holds 3 examples, rank 1 one: SyncBN normalises with the summed
    element count (it rides in the all-reduced sums), and two steps with
    broadcast initial weights match the 1-process run on the whole batch."""
    import dp_worker
    ref = dp_worker.run_cnnblstm(steps=2)
    ranks = _run_ranks("cnnblstm_uneven", tmp_path)
    assert _rel(ranks[0]["loss"], ref["loss"]) < 1e-5
    _check_state(ranks, ref, tol=1e-4)


@pytest.mark.timeout(300)
def test_gan_dp2_faithful_g_backward_two_steps(tmp_path):
    """faithful_g_backward=True under DP: the G-step backward's D gradients do
    not enter the reducer (no 'ready twice' on the next step) and two steps
    match the 1-process run."""
    import dp_worker
    ref = dp_worker.run_gan(faithful=True, steps=2)
    ranks = _run_ranks("gan_faithful", tmp_path)
    for k, v in ref["disc"].items():
        assert _rel(ranks[0]["disc"][k], v) < 1e-4, k


@pytest.mark.timeout(300)
def test_gan_dp2_fix_generator_grad_equals_single_process(tmp_path):
    """fix_generator_grad under DP: G's exchanged gradients equal the
    1-process gradients of the whole batch.  Pins the two scale conventions
    of the DP generator backward: the L1 terms are global-batch
    values (their per-rank gradient is pre-scaled for the reducer's average)
    and SyncBN's dgamma / dbeta come from all-reduced sums (handed over as the
    per-rank share)."""
    import dp_worker
    ref = dp_worker.run_gan(fix_g=True)
    ranks = _run_ranks("gan_fixg", tmp_path)
    assert set(ranks[0]["gen_grad"]) == set(ref["gen_grad"])
    for k, v in ref["gen_grad"].items():
        assert _rel(ranks[0]["gen_grad"][k], v) < 1e-3, k
        assert torch.equal(ranks[0]["gen_grad"][k], ranks[1]["gen_grad"][k]), k
    for k, v in ref["gen"].items():
        if v.is_floating_point():
            assert _rel(ranks[0]["gen"][k], v) < 1e-4, k


@pytest.mark.timeout(300)
def test_gan_dp2_nonfinite_g_loss_fails_fast_on_every_rank(tmp_path):
    """faithful_g_backward with fail_fast: a NaN G-step loss on rank 1 stops
    both ranks before g_optimizer.step() (MAX-all-reduced flag)."""
    ranks = _run_ranks("gan_gnan", tmp_path)
    assert "G loss" in ranks[1]["error"] and "on this rank" in ranks[1]["error"]
    assert "G loss" in ranks[0]["error"] and "another DP rank" in ranks[0]["error"]


@pytest.mark.timeout(300)
def test_gan_dp2_equals_single_process(tmp_path):
    import dp_worker
    ref = dp_worker.run_gan()
    ranks = _run_ranks("gan", tmp_path)
    for k, v in ref["losses"].items():
        assert abs(float(ranks[0]["losses"][k]) - float(v)) <= 1e-5 * max(1.0, abs(float(v))), k
        assert float(ranks[0]["losses"][k]) == float(ranks[1]["losses"][k]), k
    for k, v in ref["disc"].items():
        assert _rel(ranks[0]["disc"][k], v) < 1e-5, k
        assert torch.equal(ranks[0]["disc"][k], ranks[1]["disc"][k]), k
    for k, v in ref["gen_bn"].items():      # SyncBN: running stats of the global batch
        assert _rel(ranks[0]["gen_bn"][k], v) < 1e-5, k
