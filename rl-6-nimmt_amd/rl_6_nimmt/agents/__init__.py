"""Agents on the hot path (reference registry: rl_6_nimmt/agents/__init__.py:33-53).

Kept: Agent, DrunkHamster ("random"), MCSAgent ("mcts").  The model-free
learners (DQN / ACER / REINFORCE), the human UI and the PUCT variants are
outside this build's scope; their registry keys map to
`None` so scripts fail with a clear message instead of a missing key.
"""
from .base import Agent
from .random import DrunkHamster
from .mcts import BaseMCAgent, MCSAgent

HUMAN = "human"
RANDOM_AGENT = "random"
MCS = "mcts"
PMCS = "pmcs"
PUCT = "puct"

AGENTS = {
    RANDOM_AGENT: DrunkHamster,
    MCS: MCSAgent,
}
