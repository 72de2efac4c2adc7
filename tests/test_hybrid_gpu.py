"""Tensor x pipeline parallel GPT on the HIP device: two ranks sharing the one GPU of
the test box (gloo process group; pipeline activations staged through the host),
TP2 and PP2 layouts, against the single-process fp32 reference of
tests/hybrid_common.py (the 8-rank TP2 x PP2 x sharding-3 composition is
tests/test_hybrid_cpu.py)."""
import pytest

from dist_util import run_dist
from hybrid_common import M, check, reference, worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mp_deg,pp_deg", [(2, 1), (1, 2)], ids=["tp2", "pp2"])
def test_gpt_tp_pp_two_ranks_one_gpu_match_single_process(mp_deg, pp_deg):
    ref_losses, init, ref_final = reference(M, paddle_eps=True)
    res = run_dist(worker, 2, init, mp_deg, pp_deg, 1, "cuda", timeout=400)
    check(res, ref_losses, ref_final, loss_tol=2e-4, atol=2e-4)
