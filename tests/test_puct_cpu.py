"""Host logic of the config-4 rollout MLP (no GPU): FusedMLP's one-kernel
form (the tensors sn_puct_mlp_seats / sn_puct_rollouts read) -- layer 1 per
seat through the [W1 | b1 | 0] rows of w1s with the ones feature, the card
column w1c added per candidate, layer 2 through [W2 | b2 | 0] with the ones
pass-through row, the head [wh | bh | 0] -- restates the module's own
forward on the full [card, obs] rows; other layouts get no fused form; and
refresh_from copies new weights into the same tensors (the captured
hipGraphs stay valid)."""
import torch

from rl_6_nimmt.puct import FusedMLP, make_actor
from rl_6_nimmt.utils.nets import MultiHeadedMLP


def _fused_forward(fz, obs, cards, n_cur):
    """the kernels' arithmetic in f32, without their bf16 roundings of the
    activations: what the padded tensors encode"""
    w1c, w2p, head, w1s = (t.float() for t in fz)
    S = obs.shape[0]
    seat = torch.zeros((S, 64))
    seat[:, 1:48] = obs
    seat[:, 48] = 1.0  # the ones feature
    base = seat @ w1s.t()  # [S, 128]: rows >= H are 0 except the ones row H
    h1 = torch.relu(base[:, :112].repeat_interleave(n_cur, dim=0) + cards[:, None] * w1c[None, :])
    h2 = torch.relu(h1 @ w2p.t())  # [R, 128]: the ones pass-through row H2 carries the head bias
    return h2 @ head


def test_fused_form_restates_module_forward():
    torch.manual_seed(0)
    net = make_actor().to(torch.bfloat16)
    fm = FusedMLP.of(net)
    fz = fm.fused()
    assert fz is not None
    w1c, w2p, head, w1s = fz
    assert w1c.shape == (112,) and w2p.shape == (128, 112) and head.shape == (128,) and w1s.shape == (128, 64)
    assert float(w1s[100, 48]) == 1.0 and float(w2p[100, 100]) == 1.0  # ones feature / pass-through
    S, n_cur = 37, 5
    obs = (torch.rand(S, 47) * 2 - 1).to(torch.bfloat16).float()
    cards = (torch.rand(S * n_cur) * 2 - 1).to(torch.bfloat16).float()
    rows = torch.cat((cards[:, None], obs.repeat_interleave(n_cur, dim=0)), dim=1)  # [R, 48]
    with torch.no_grad():
        (want,) = net.float()(rows)
    got = _fused_forward(fz, obs, cards, n_cur)
    assert torch.allclose(got, want[:, 0], rtol=1e-5, atol=1e-5)


def test_fused_form_rejects_other_layouts():
    torch.manual_seed(0)
    relu = torch.nn.ReLU()
    for net in (MultiHeadedMLP(47, hidden_sizes=(32, 32), head_sizes=(1,), activation=relu,
                               head_activations=(None,)).to(torch.bfloat16),   # another input width
                MultiHeadedMLP(48, hidden_sizes=(40, 24, 16), head_sizes=(1,), activation=relu,
                               head_activations=(None,)).to(torch.bfloat16),   # three hidden layers
                make_actor()):                                                 # fp32
        assert FusedMLP.of(net).fused() is None  # these run sn_puct_rows + the module's forward


def test_refresh_from_updates_in_place():
    torch.manual_seed(1)
    actor = make_actor().to(torch.bfloat16)
    net = FusedMLP.of(make_actor().to(torch.bfloat16))
    net.refresh_from(actor)
    fz = net.fused()
    before = [t.data_ptr() for t in fz] + [net.head_w.data_ptr(), net.head_b.data_ptr()]
    with torch.no_grad():
        for p in actor.parameters():
            p.add_(0.25)
    assert net.refresh_from(actor)
    after = [t.data_ptr() for t in net.fused()] + [net.head_w.data_ptr(), net.head_b.data_ptr()]
    assert before == after
    fresh = FusedMLP.of(actor)
    for a, b in zip(net.fused(), fresh.fused()):
        assert torch.equal(a, b)
    assert torch.equal(net.head_w, fresh.head_w) and torch.equal(net.head_b, fresh.head_b)
    other = MultiHeadedMLP(48, hidden_sizes=(64,), head_sizes=(1,), activation=torch.nn.ReLU(), head_activations=(None,))
    assert not net.refresh_from(other)
