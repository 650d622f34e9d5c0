"""Paths of albedo's date-keyed caches (settings/package.scala:8-19).

`spark.albedo.dataDir` / `spark.albedo.checkpointDir` (SparkConf keys, defaults ./spark-data and
./spark-data/checkpoint) become the environment variables ALBEDO_DATA_DIR / ALBEDO_CHECKPOINT_DIR;
`today` is the yyyyMMdd key of the caches.
"""
from __future__ import annotations

import datetime
import os


def data_dir() -> str:
    return os.environ.get("ALBEDO_DATA_DIR", "./spark-data")


def checkpoint_dir() -> str:
    return os.environ.get("ALBEDO_CHECKPOINT_DIR", "./spark-data/checkpoint")


def today() -> str:
    return datetime.datetime.now().strftime("%Y%m%d")


def als_model_path() -> str:
    """ALSRecommenderBuilder.scala:44 / ALSRecommender.scala:17."""
    return f"{data_dir()}/{today()}/alsModel.parquet"


def raw_starring_path() -> str:
    """DatasetUtils.scala:114 (loadRawStarringDS's parquet cache)."""
    return f"{data_dir()}/{today()}/rawStarringDF.parquet"
