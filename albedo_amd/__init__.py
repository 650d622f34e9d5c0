"""albedo_amd — MI355X-native implicit-ALS candidate generation (drop-in for the Spark ML ALS path
of land1725/albedo: ALSRecommenderBuilder -> ALS.fit -> ALSRecommender top-k -> NDCG@30).

Layout:
  csrc/           HIP kernels (gfx950) + the C ABI engine -> libalbedo_als.so (include/albedo_als.h)
  _lib.py         ctypes binding of the C ABI
  als.py          Spark-shaped ALS / ALSModel facade
  evaluation.py   RankingEvaluator / ndcgAt (RankingEvaluator.scala:83-139)
  recommenders.py Recommender / ALSRecommender transformers (recommenders/*.scala)
  builder.py      ALSRecommenderBuilder.main + loadOrCreateModel (ModelUtils.scala:7-20)
  settings.py     dataDir / checkpointDir / today (settings/package.scala)
  synthetic.py    seeded power-law star matrices (BASELINE configs)
"""
from .als import ALS, ALSModel, SPARK_DEFAULT_SEED  # noqa: F401
from ._lib import ALSError, IllegalArgumentException, IllegalStateException  # noqa: F401
from .evaluation import RankingEvaluator  # noqa: F401
from .recommenders import ALSRecommender, Recommender  # noqa: F401

__all__ = ["ALS", "ALSModel", "ALSError", "IllegalArgumentException", "IllegalStateException",
           "SPARK_DEFAULT_SEED", "RankingEvaluator", "Recommender", "ALSRecommender"]
