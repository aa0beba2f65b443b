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


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_clip_handoff_matches_in_place_clip(device):
    """clip_grad_norm_(..., optimizer=adam) on an arena-backed model leaves the gradient scaling to
    Adam's kernel (stored back while it reads g).  Parameters, moments AND the gradients after step()
    must equal the separate in-place clip followed by an unscaled Adam step, bit for bit."""
    import copy

    from deeplearning_mpi_amd.models import resnet18
    from deeplearning_mpi_amd.ops import cross_entropy

    torch.manual_seed(0)
    m1 = resnet18(num_classes=10).to(device)
    m2 = copy.deepcopy(m1)
    x = torch.randn(4, 3, 32, 32, device=device)
    y = torch.tensor([1, 7, 3, 0], device=device)
    out = []
    for m, handoff in ((m1, True), (m2, False)):
        opt = Adam(m.parameters(), lr=1e-3)
        for _ in range(2):
            opt.zero_grad()
            cross_entropy(m(x), y).backward()
            if handoff:
                clip_grad_norm_(m.parameters(), 0.05, optimizer=opt)
                assert opt._clip_handoff
            else:
                clip_grad_norm_(m.parameters(), 0.05)   # scales in place
            opt.step()
            assert opt.clip is None
        out.append(([p.detach().clone() for p in m.parameters()], [p.grad.detach().clone() for p in m.parameters()]))
    for a, b in zip(out[0][0] + out[0][1], out[1][0] + out[1][1]):
        assert torch.equal(a, b)
