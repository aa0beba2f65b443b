"""Adam after a collectively skipped step (non-finite gradient norm) must be exactly the run that
never had that step: parameters, moments AND the device step count behind the bias corrections
(the count used to advance on skipped steps).  CPU (reference backend) always; the
fused gfx950 kernels when a GPU is present."""
import pytest
import torch

from deeplearning_mpi_amd.optim import Adam, clip_grad_norm_


def _run(grads, device):
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(1000, device=device))
    opt = Adam([p], lr=1e-2)
    for g in grads:
        opt.zero_grad()
        p.grad = g.to(device).clone()
        clip_grad_norm_([p], 1.0, optimizer=opt)
        opt.step()
    st = opt.state[p]
    return p.detach().cpu(), st["exp_avg"].cpu(), st["exp_avg_sq"].cpu(), float(st["step"].reshape(-1)[0])


def _grads():
    g = torch.Generator().manual_seed(1)
    return [torch.randn(1000, generator=g) * s for s in (0.5, 3.0, 0.2)]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_adam_skipped_step_is_a_no_op(device):
    g1, g2, g3 = _grads()
    bad = g2.clone()
    bad[7] = float("nan")
    with_skip = _run([g1, bad, g2, g3], device)
    without = _run([g1, g2, g3], device)
    assert with_skip[3] == without[3] == 3.0
    for a, b in zip(with_skip[:3], without[:3]):
        assert torch.equal(a, b)
