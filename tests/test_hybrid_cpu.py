"""Composed hybrid parallelism (BASELINE config 4 shape: GPT-3, TP x PP x sharding
stage 3) on 8 gloo ranks = TP2 x PP2 x sharding 2, against ONE process training the
same model on the same global batch with an fp32 AdamW + global-norm clip reference.

fleet.distributed_model builds the pipeline stages of tensor-parallel GPT blocks and
wraps each stage's blocks as ZeRO-3 gather-on-use units on the sharding axis (tied
embedding kept whole, summed across the two stages); HybridParallelOptimizer hands
lr / betas / eps / clip to the sharded engine.  Reference seed of the sharding side:
framework/details/multi_devices_graph_pass.cc:247 (GetAppropriateDeviceID), :412-452.
"""
import pytest

from dist_util import run_dist
from hybrid_common import M, check, reference, worker


@pytest.mark.timeout(600)
def test_gpt_tp2_pp2_sharding3_matches_single_process():
    # 2 sharding ranks x M micro-batches, equal sizes: mean over 2M micro-batch losses
    ref_losses, init, ref_final = reference(2 * M)
    res = run_dist(worker, 8, init, 2, 2, 2, "cpu")
    check(res, ref_losses, ref_final, loss_tol=2e-5, atol=2e-5)
