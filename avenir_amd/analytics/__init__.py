"""Analytics: data exploration, PCA, time-series generation, model interpretation."""
from .explorer import DataExplorer
from .interpret import LimeTabular, ice_grid, individual_conditional_expectation, partial_dependence
from .pca import PCA, IncrementalPCA, PrincipalCompState
from .timeseries import TimeSeriesGenerator
