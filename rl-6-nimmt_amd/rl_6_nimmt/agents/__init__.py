"""Agents on the hot path (reference registry: rl_6_nimmt/agents/__init__.py:33-53).

Kept: Agent, DrunkHamster ("random"), MCSAgent ("mcts"), PolicyMCSAgent
("pmcs"), PUCTAgent ("puct"), BatchedReinforceAgent ("reinforce") and
PUCTCustomedAgent (exported, not in the registry -- as in the reference).
The other model-free learners (DQN family, ACER) and the human UI are
outside this build's scope and absent from AGENTS.
"""
from .base import Agent
from .random import DrunkHamster
from .mcts import BaseMCAgent, MCSAgent, PolicyMCSAgent, PUCTAgent, PUCTCustomedAgent
from .policy import BatchedReinforceAgent

HUMAN = "human"
RANDOM_AGENT = "random"
REINFORCE = "reinforce"
MCS = "mcts"
PMCS = "pmcs"
PUCT = "puct"

AGENTS = {
    RANDOM_AGENT: DrunkHamster,
    REINFORCE: BatchedReinforceAgent,
    MCS: MCSAgent,
    PMCS: PolicyMCSAgent,
    PUCT: PUCTAgent,
}
