"""Configuration with the keys the reference's hot path reads (reference const.py:11-518):
``cfg.DATA_SET``, ``cfg.MODEL["name" | "HyperParameter" | "save_path"]``,
``cfg.RECOMMEND["k" | "save_path" | "target_user"]``, ``cfg.LOG``, ``cfg.PREPROCESSING[...]``
(every key of the reference's, including the ETL keys ``dataset_path_dict``, ``columns_map``,
``quantile`` and ``vector_size`` that main.py's cache-miss branch and processing/* read).

Selection is by environment variables instead of editing module globals
(reference const.py:494-518): LGCNHS_ENV (dev|prod), LGCNHS_DATASET (movielens|douban),
LGCNHS_MODEL, LGCNHS_ROOT (output root, default ./RS/algorithm/temp). Two deliberate
differences: no directories are created at import (they are made when a file is saved),
and the dev environment also defines LightGCNOpti / SpreadLightGCNOpti, which the
reference's DevConfig lacks (its default configuration cannot run).
"""
from __future__ import annotations

import os

_TRAIN = {"seed": 42, "embedding_dim": 64, "layers": 3, "lr": 1e-3, "gamma": 0.95,
          "epoch_per_eval": 200, "epoch_per_lr_decay": 200, "batch_size": 1024,
          "epsilon": 1e-6}

# (env, model) -> hyper-parameters; values from reference const.py:111-177 (dev) and
# :305-421 (prod)
_HP = {
    ("dev", "ProbS"): {"lambda": 1},
    ("dev", "HeatS"): {"lambda": 0},
    ("dev", "HybridS"): {"lambda": 0.3},
    ("dev", "LightGCN"): dict(_TRAIN, epochs=10),
    ("dev", "LightGCNOpti"): dict(_TRAIN, epochs=10),
    ("dev", "SpreadLightGCN"): dict(_TRAIN, epochs=10, **{"lambda": 0.5}),
    ("dev", "SpreadLightGCNOpti"): dict(_TRAIN, epochs=10, **{"lambda": 0.5}),
    ("prod", "ProbS"): {"lambda": 1},
    ("prod", "HeatS"): {"lambda": 0},
    ("prod", "HybridS"): {"lambda": 0.6},
    ("prod", "LightGCN"): dict(_TRAIN, epochs=10000),
    ("prod", "LightGCNOpti"): dict(_TRAIN, epochs=10000),
    ("prod", "SpreadLightGCN"): dict(_TRAIN, epochs=10000, **{"lambda": 0.85}),
    ("prod", "SpreadLightGCNOpti"): dict(_TRAIN, epochs=10000, **{"lambda": 0.6}),
}


# per-dataset ETL keys (reference const.py:81-95 defaults, :202-244 dev, :446-488 prod)
_DATASET_DIRS = {("dev", "movielens"): "I:/Workspace/data/ml-100k/",
                 ("dev", "douban"): "I:/Workspace/data/douban/",
                 ("prod", "movielens"): "/data/datasets/recommend/ml-100k/",
                 ("prod", "douban"): "/data/datasets/recommend/douban/"}
_ETL = {
    "movielens": {
        "files": {"users": "u.user", "items": "u.item", "rating": "u.data",
                  "occupation": "u.occupation"},
        "columns_map": {"user_id": "user", "item_id": "item", "rating": "rating",
                        "rating_time": "timestamp"},
        "quantile": {"start": 1, "end": 0},
        "vector_size": {"title": 5, "content": 20},
    },
    "douban": {
        "files": {"users": "users.csv", "items": "movies.csv", "rating": "ratings.csv"},
        "columns_map": {"user_id": "USER_MD5", "item_id": "MOVIE_ID", "rating": "RATING",
                        "rating_time": "RATING_TIME"},
        "quantile": {"start": 0.991, "end": 0.99},
        "vector_size": {"title": 3, "content": 20},
        "target_user": "1a76e2591cd2f3740ccb7f198dace22a",
    },
}


class Config:
    def __init__(self, env: str = "dev", dataset: str = "movielens",
                 model: str = "SpreadLightGCNOpti", root: str | None = None) -> None:
        if root is None:
            root = "./RS/algorithm/temp" if env == "dev" else "/data/alex/algorithm"
        base = os.path.join(root, dataset)
        self.ENV = env
        self.DATA_SET = dataset
        etl = _ETL.get(dataset, {})
        ddir = _DATASET_DIRS.get((env, dataset), "")
        self.PREPROCESSING = {
            "seed": 42,
            "dataset_path_dict": {k: ddir + f for k, f in etl.get("files", {}).items()},
            "save_path": base + "/preprocess/",
            "vector_size": dict(etl.get("vector_size", {})),
            "columns_map": dict(etl.get("columns_map", {})),
            "quantile": dict(etl.get("quantile", {"start": 1, "end": 0})),
            "split_percentage": [0.2, 0.5],
        }
        self.LOG = {"file_path": base + "/log/"}
        self.MODEL = {"name": model, "HyperParameter": dict(_HP.get((env, model), {})),
                      "save_path": base + "/model/"}
        self.EVALUATION = {"save_path": base + "/evaluation/"}
        self.RECOMMEND = {"k": 10 if env == "dev" else 100, "save_path": base + "/recommend/"}
        if "target_user" in etl:
            self.RECOMMEND["target_user"] = etl["target_user"]
        self.PICTURES = {"save_path": base + "/pictures/"}


cfg = Config(os.environ.get("LGCNHS_ENV", "dev"), os.environ.get("LGCNHS_DATASET", "movielens"),
             os.environ.get("LGCNHS_MODEL", "SpreadLightGCNOpti"), os.environ.get("LGCNHS_ROOT"))
