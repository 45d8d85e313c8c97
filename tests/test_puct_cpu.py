"""Host logic of the config-4 rollout MLP (no GPU): FusedMLP's feature-major
split form -- per-seat layer 1 through [W1 | b1 | 0], the card column added
per candidate (what k_puct_h1_cols computes), the later layers and the head
as augmented GEMMs with the biases riding on a ones feature -- equals the
module's own forward on the full [card, obs] rows; and refresh_from copies
new weights into the same tensors (the captured hipGraphs stay valid)."""
import pytest
import torch

from rl_6_nimmt.puct import FusedMLP, make_actor
from rl_6_nimmt.utils.nets import MultiHeadedMLP


def _h1_cols(base, cards, w1c, n_cur, kp):
    """k_puct_h1_cols on the host: h1T[j][r] = relu(baseT[j][r // n_cur] +
    cards[r] * w1c[j]) for j < H, 1 at j = H, 0 up to kp"""
    H, S = base.shape
    R = S * n_cur
    seat = torch.arange(R) // n_cur
    h = torch.relu(base[:, seat] + cards[None, :] * w1c[:, None])
    out = torch.zeros((kp, R), dtype=base.dtype)
    out[:H] = h
    out[H] = 1
    return out


@pytest.mark.parametrize("hidden", [(100, 100), (64,), (40, 24, 16)])
def test_feature_major_split_equals_module_forward(hidden):
    torch.manual_seed(0)
    net = MultiHeadedMLP(48, hidden_sizes=hidden, head_sizes=(1,), activation=torch.nn.ReLU(), head_activations=(None,))
    fm = FusedMLP.of(net)
    w1a, H, kp, layers, ha, w1c = fm.split()
    assert H == hidden[0] and kp % 8 == 0 and kp > H
    S, n_cur = 37, 5
    obs = torch.rand(S, 47) * 2 - 1
    cards = torch.rand(S * n_cur) * 2 - 1
    rows = torch.cat((cards[:, None], obs.repeat_interleave(n_cur, dim=0)), dim=1)  # [R, 48]
    cols = torch.zeros((56, S))
    cols[1:48] = obs.t()
    cols[48] = 1
    base = w1a @ cols
    x = _h1_cols(base, cards, w1c, n_cur, kp)
    for wa in layers:
        x = torch.relu(wa @ x)
    out = (ha @ x)[0]
    with torch.no_grad():
        (want,) = net(rows)
    assert torch.allclose(out, want[:, 0], rtol=1e-5, atol=1e-5)


def test_split_rejects_other_layouts():
    torch.manual_seed(0)
    net = MultiHeadedMLP(47, hidden_sizes=(32,), head_sizes=(1,), activation=torch.nn.ReLU(), head_activations=(None,))
    assert FusedMLP.of(net).split() is None


def test_refresh_from_updates_in_place():
    torch.manual_seed(1)
    actor = make_actor()
    net = FusedMLP.of(make_actor())
    net.refresh_from(actor)
    before = [t.data_ptr() for t in net._split_tensors()] + [net.head_w.data_ptr(), net.head_b.data_ptr()]
    with torch.no_grad():
        for p in actor.parameters():
            p.add_(0.25)
    assert net.refresh_from(actor)
    after = [t.data_ptr() for t in net._split_tensors()] + [net.head_w.data_ptr(), net.head_b.data_ptr()]
    assert before == after
    fresh = FusedMLP.of(actor)
    for a, b in zip(net._split_tensors(), fresh._split_tensors()):
        assert torch.equal(a, b)
    assert torch.equal(net.head_w, fresh.head_w) and torch.equal(net.head_b, fresh.head_b)
    other = MultiHeadedMLP(48, hidden_sizes=(64,), head_sizes=(1,), activation=torch.nn.ReLU(), head_activations=(None,))
    assert not net.refresh_from(other)
