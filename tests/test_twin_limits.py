"""CPU check: the twin update's eligibility caps (mjx_amd/twin.py) equal the fused launches' capacities
in the kernel source (csrc/ppo_loss_kernels.hip), so a net too deep for mjl_adam_multi /
mjl_slice_sum_multi is never routed to the twin path."""
import os
import re

from mjx_amd import twin

SRC = os.path.join(os.path.dirname(__file__), "..", "mujoco-mjx-lab_amd", "csrc", "ppo_loss_kernels.hip")


def _const(name):
    m = re.search(r"constexpr int %s = (\d+);" % name, open(SRC).read())
    assert m, name
    return int(m.group(1))


def test_twin_caps_match_kernel_capacities():
    assert twin.ADAM_MULTI_MAX_T == _const("kAdamMultiMaxT")
    assert twin.SLICE_SEG_MAX == _const("kSliceSegMax")
    # the reference's 3 x 256 nets (nl = 4) fit; 5 hidden layers (nl = 6) do not
    assert 4 * 4 + 1 <= twin.ADAM_MULTI_MAX_T and 2 * 4 + 2 <= twin.SLICE_SEG_MAX
    assert 4 * 6 + 1 > twin.ADAM_MULTI_MAX_T
