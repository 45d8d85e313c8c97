"""Agents on the hot path (reference registry: rl_6_nimmt/agents/__init__.py:33-53).

Kept: Agent, DrunkHamster ("random"), MCSAgent ("mcts"), PolicyMCSAgent
("pmcs"), PUCTAgent ("puct").  The model-free
learners (DQN / ACER / REINFORCE), the human UI and PUCTCustomedAgent are
outside this build's scope and absent from AGENTS.
"""
from .base import Agent
from .random import DrunkHamster
from .mcts import BaseMCAgent, MCSAgent, PolicyMCSAgent, PUCTAgent

HUMAN = "human"
RANDOM_AGENT = "random"
MCS = "mcts"
PMCS = "pmcs"
PUCT = "puct"

AGENTS = {
    RANDOM_AGENT: DrunkHamster,
    MCS: MCSAgent,
    PMCS: PolicyMCSAgent,
    PUCT: PUCTAgent,
}
