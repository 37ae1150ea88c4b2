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
