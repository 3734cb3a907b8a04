"""The device update path pinned to the reference's PPO at BASELINE C2 size (tests/golden/make_golden_ppo_c2.py:
standalone/rsl_rl/ext/algorithms/ppo.py:103-190 over plain nn.Linear layers, 4 096 envs x 24 steps, 24 576-row
mini-batches): on cuda:0 the update runs TallLinear's split-K weight gradients and gr_column_sum bias gradients,
eager and graph-captured (one graph per mini-batch step, one per epoch, and the two-segment form used at world size > 1)
with capturable Adam.  Pins and
tolerances: tests/ppo_c2_golden.py."""
import pytest

import ppo_c2_golden as pc2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gp():
    return pc2.load()


@pytest.mark.parametrize("opts", [dict(), dict(graph_update=True, graph_update_per_step=True), dict(graph_update=True),
                                  dict(graph_update=True, graph_update_segmented=True)],
                         ids=["eager", "graphed_per_step", "graphed_epoch", "graphed_segmented"])
def test_device_update_matches_reference_c2(gp, opts):
    rep = pc2.replay(gp, "cuda:0", **opts)
    print(opts, rep)
