"""Application-level simulations of the reference's ``P/app`` drivers, on the framework's device
samplers and estimators: project-cost confidence bounds (pccb.py), MCMC inventory planning
(inv_sim.py) and the manufacturing back-order causal model (back_order.py)."""
from .inventory import InventorySimulation
from .project_cost import ProjectCostModel, project_cost_simulation
from .supply import SupplyChainSimulation, back_order_intervention

__all__ = ["InventorySimulation", "ProjectCostModel", "project_cost_simulation", "SupplyChainSimulation",
           "back_order_intervention"]
