"""avenir_amd — an MI355X-native (CDNA4 / gfx950) predictive-analytics framework with the
capabilities of the avenir toolkit (Naive Bayes, trees/forests, KNN, clustering, SVM, regression,
Markov/HMM, association mining, bandits, optimisers, Monte-Carlo, small neural models, text and
exploratory analytics).

Layers: ``utils`` (config, schema, logging, metrics, checkpoint, tracing),
``data`` (CSV -> device columns), ``parallel`` (RCCL collectives), ``ops`` (HIP kernel wrappers),
``models`` (estimators), ``optimize``, ``nn``, ``text``, ``analytics``, ``cli`` and ``serve`` (surfaces).
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401


def freeze_startup_objects() -> None:
    """Opt-in for entry points (CLI, bench, smoke): move every object alive now (torch, numpy,
    this package: several hundred thousand) to the GC's permanent generation, so a generation-2
    collection triggered by model code that builds many small Python objects no longer walks them
    (such a pass cost 50-100 ms in the middle of a 20 ms forest build).  Importing the library
    never does this — an embedding application keeps its own GC behaviour.  AVMI_GC_FREEZE=0
    disables it."""
    import gc
    import os
    if os.environ.get("AVMI_GC_FREEZE", "1") != "0" and hasattr(gc, "freeze"):
        gc.collect()
        gc.freeze()
