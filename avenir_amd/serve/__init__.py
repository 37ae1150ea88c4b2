"""Serving surfaces: REST prediction service with micro-batching, online bandit service."""
from .bandit_service import BanditService, simulate_lead_generation
from .rest import MicroBatcher, PredictionServer, classifier_factory, parse_recs
