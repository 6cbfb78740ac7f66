"""Diagnostic: forward + backward of the update's Gaussian log-prob ([65536, 21]) through autograd
of the elementwise formula vs the hand-written backward (ppo._GaussianLogprob). Not product code."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mujoco-mjx-lab_amd"))
import torch  # noqa: E402

from mjx_amd import ppo  # noqa: E402


def plain(mean, ls, act):
    var = torch.exp(2.0 * ls)
    return torch.sum((act - mean) ** 2 / var + 2.0 * ls + ppo.LOG2PI, dim=-1) * -0.5


g = torch.Generator(device="cuda").manual_seed(0)
mean = torch.randn((65536, 21), generator=g, device="cuda").requires_grad_()
ls = (0.3 * torch.randn(21, generator=g, device="cuda")).requires_grad_()
act = torch.randn((65536, 21), generator=g, device="cuda")
gout = torch.randn(65536, generator=g, device="cuda")
for name, f in (("autograd", plain), ("custom", ppo._GaussianLogprob.apply)):
    def step():
        return torch.autograd.grad(f(mean, ls, act), (mean, ls), gout)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(50):
        r = step()
    torch.cuda.synchronize()
    print(name, "%.1f us per fwd+bwd" % ((time.time() - t) / 50 * 1e6), flush=True)
a, b = plain(mean, ls, act), ppo._GaussianLogprob.apply(mean, ls, act)
ga, gb = torch.autograd.grad(a, (mean, ls), gout), torch.autograd.grad(b, (mean, ls), gout)
print("max |logp diff| %.2e, |dmean| %.2e, |dlog_std| %.2e (rel %.2e)" % (
    float((a - b).abs().max()), float((ga[0] - gb[0]).abs().max()), float((ga[1] - gb[1]).abs().max()),
    float((ga[1] - gb[1]).abs().max() / ga[1].abs().max())))
