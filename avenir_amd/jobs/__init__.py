"""CLI job layer: one registered function per reference MR / Spark job, external pipeline stage
and Python driver (see ``python -m avenir_amd --list``)."""
from .common import JOBS, JobContext, job  # noqa: F401
from . import app_jobs, app_more_jobs, core, explore_jobs, markov_jobs, model_jobs, pipeline_stages, text_jobs  # noqa: F401,E402
