"""Stochastic optimisation (reference J/optimize, S/optimize, P/mlextra/opti*.py): batched search
domains and population / multi-chain optimisers on device tensors."""
from .domain import AssignmentDomain, CallbackDomain, FunctionDomain, SearchDomain
from .domains import FeatureSubsetDomain, MeetingScheduleDomain, TaskScheduleSearch, geo_distance, read_lenient_json
from .search import (BayesianOptimizer, EvolutionaryOptimizer, GeneticAlgorithm, OptResult, RandomSearch,
                     SimulatedAnnealing, TabuSearch, local_focussed, local_trajectory, parameter_search, sa_assign,
                     sa_assign_reference)

__all__ = [
    "AssignmentDomain", "CallbackDomain", "FunctionDomain", "SearchDomain", "FeatureSubsetDomain",
    "MeetingScheduleDomain", "TaskScheduleSearch", "geo_distance", "read_lenient_json", "BayesianOptimizer",
    "EvolutionaryOptimizer", "GeneticAlgorithm", "OptResult", "RandomSearch", "SimulatedAnnealing", "TabuSearch",
    "local_focussed", "local_trajectory", "parameter_search", "sa_assign", "sa_assign_reference",
]
