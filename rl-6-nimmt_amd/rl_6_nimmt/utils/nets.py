"""Policy network of the MCS/PUCT agents (reference: rl_6_nimmt/utils/nets.py:100-132).

`MultiHeadedMLP(input, hidden_sizes, head_sizes, activation, head_activations)`
with the reference's module layout (`latent_net.<i>`, `head_nets.<h>.0`), so
state_dicts are interchangeable with the reference's.  The noisy/duelling
DQN variants are out of scope.
"""
from torch import nn


class MultiHeadedMLP(nn.Module):
    def __init__(self, input_size, hidden_sizes, head_sizes, activation, head_activations, linear=nn.Linear,
                 init_sigma=1.0):
        super().__init__()
        if linear is not nn.Linear:
            raise NotImplementedError("noisy layers are outside this build's scope")
        layers, width = [], input_size
        for h in hidden_sizes:
            layers += [linear(width, h), activation]
            width = h
        self.latent_net = nn.Sequential(*layers)
        self.head_nets = nn.ModuleList()
        for size, act in zip(head_sizes, head_activations):
            head = [linear(width, size)] + ([act] if act is not None else [])
            self.head_nets.append(nn.Sequential(*head))

    def forward(self, inputs):
        latent = self.latent_net(inputs)
        return [head(latent) for head in self.head_nets]
