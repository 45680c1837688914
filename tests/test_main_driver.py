"""main.py's Step 1-3 sequence (reference main.py:26-106) through the package's own driver,
from preprocessed CSVs written to the configured cache directory: every model name of the
dispatch (dev config), the recommendation dict saved and reloaded on the second run, the six
test metrics in range."""
import os

import numpy as np
import pandas as pd
import pytest

MODELS = ["HybridS", "ProbS", "LightGCN", "LightGCNOpti", "SpreadLightGCN",
          "SpreadLightGCNOpti"]


def _write_cache(d, U=90, I=160, E=4000, seed=7):
    from lgcnhs.synth import synth_dataframes
    rating_df, tr, va, te = synth_dataframes(U, I, E, seed=seed, dist="zipf")
    os.makedirs(d, exist_ok=True)
    rating_df.to_csv(d + "filter_rating.csv", index=False)
    tr.to_csv(d + "train_data.csv", index=False)
    va.to_csv(d + "val_data.csv", index=False)
    te.to_csv(d + "test_data.csv", index=False)
    rng = np.random.default_rng(seed)
    pd.DataFrame({"user_id": np.arange(U),
                  "user_features": [str([round(float(x), 4) for x in rng.normal(size=8)]) for _ in range(U)]}
                 ).to_csv(d + "user_features.csv", sep="\t", index=False)
    pd.DataFrame({"item_id": np.arange(I),
                  "item_features": [str([round(float(x), 4) for x in rng.normal(size=8)]) for _ in range(I)]}
                 ).to_csv(d + "item_features.csv", sep="\t", index=False)
    return U, I


@pytest.fixture
def cache_cfg(tmp_path):
    from const import cfg
    saved = {k: dict(getattr(cfg, k)) for k in ("PREPROCESSING", "MODEL", "RECOMMEND",
                                                 "PICTURES", "EVALUATION")}
    base = str(tmp_path) + "/"
    cfg.PREPROCESSING["save_path"] = base + "preprocess/"
    cfg.MODEL["save_path"] = base + "model/"
    cfg.RECOMMEND["save_path"] = base + "recommend/"
    cfg.PICTURES["save_path"] = base + "pictures/"
    cfg.EVALUATION["save_path"] = base + "evaluation/"
    yield cfg
    for k, v in saved.items():
        getattr(cfg, k).clear()
        getattr(cfg, k).update(v)


def test_missing_cache_names_the_expected_files(cache_cfg):
    import main
    with pytest.raises(FileNotFoundError, match="filter_rating.csv"):
        main.load_preprocessed()


def test_config_has_the_etl_keys():
    from const import Config
    for env in ("dev", "prod"):
        for ds in ("movielens", "douban"):
            c = Config(env, ds, "LightGCN", root="/tmp/x")
            p = c.PREPROCESSING
            assert set(p["dataset_path_dict"]) >= {"users", "items", "rating"}
            assert set(p["columns_map"]) == {"user_id", "item_id", "rating", "rating_time"}
            assert set(p["quantile"]) == {"start", "end"} and set(p["vector_size"]) == {
                "title", "content"}
    assert Config("dev", "douban").RECOMMEND["target_user"]


def test_plot_metric_writes_png(tmp_path):
    from utils.picture import plotMetric
    out = str(tmp_path / "sub" / "m.png")
    plotMetric([0, 1, 2], [0.1, 0.3, 0.2], "iteration", "precision", "precision curves", out)
    assert os.path.getsize(out) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", MODELS)
def test_main_steps_1_to_3(cache_cfg, name):
    import main
    U, I = _write_cache(cache_cfg.PREPROCESSING["save_path"])
    from const import Config
    cache_cfg.MODEL["name"] = name
    # the named model's own hyper-parameters (the reference's config classes carry one model's)
    cache_cfg.MODEL["HyperParameter"] = dict(
        Config(cache_cfg.ENV, cache_cfg.DATA_SET, name).MODEL["HyperParameter"])
    hp = cache_cfg.MODEL["HyperParameter"]
    if "epochs" in hp:
        hp.update(epochs=3, epoch_per_eval=2)
    k = cache_cfg.RECOMMEND["k"]
    r1 = main.main()
    assert r1["users"] == U and r1["items"] == I
    recs = r1["recommendations"]
    assert sorted(recs) == list(range(U))
    assert all(len(v) == k and len(set(v)) == k for v in recs.values())
    for m in ("precision", "recall", "f1", "ndcg", "H", "I"):
        assert 0.0 <= float(r1[m]) <= 1.0, (m, r1[m])
    # the recommenders save under the reference's names (reference recommend.py: "_" + k,
    # except LightGCNOpti's); main's Step 2 loads "<name><k>.npy" as the reference's main.py
    # does (reference main.py:62), so only LightGCNOpti's cache hits -- the others recompute,
    # on the cached model where there is one: the second run repeats the lists either way
    sep = "" if name == "LightGCNOpti" else "_"
    path = (cache_cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + name + sep +
            str(k) + ".npy")
    assert os.path.exists(path)
    r2 = main.main()
    assert r2["recommendations"] == recs
    assert r2["precision"] == r1["precision"] and r2["H"] == r1["H"]
