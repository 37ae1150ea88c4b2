"""Neural models on PyTorch-ROCm (reference P/supv/tnn.py, lstm.py, P/unsupv/ae.py, rbm.py,
P/app/price_rl.py)."""
from .common import GraphedStep, create_activation, create_loss, create_optimizer, load_checkpoint, save_checkpoint
from .mlp import FeedForwardNetwork, parse_layer_spec
from .rl import DQNAgent, PolicyServer, PricingEnv, PricingParams, QNetwork
from .sequence import LstmNetwork
from .unsupervised import AutoEncoder, RestrictedBoltzmannMachine

__all__ = ["GraphedStep", "create_activation", "create_loss", "create_optimizer", "load_checkpoint",
           "save_checkpoint", "FeedForwardNetwork", "parse_layer_spec", "DQNAgent", "PolicyServer", "PricingEnv",
           "PricingParams", "QNetwork", "LstmNetwork", "AutoEncoder", "RestrictedBoltzmannMachine"]
