"""Entry point with the reference's three steps (reference main.py:26-106): load the
preprocessed CSV cache, run (or reload) the configured model's recommendations, evaluate
them on the test split. Same file names, same dispatch on ``cfg.MODEL["name"]``, same log
lines; the recommenders and metrics are this package's GPU paths.

Dataset ETL (the reference's processing/) is out of scope: on a cache miss
the reference's own ``processing`` package is used if it is importable, otherwise a clear
error names the CSVs that are expected under ``cfg.PREPROCESSING["save_path"]``."""
from __future__ import annotations

import pandas as pd

from const import cfg
from lgcnhs.recs import CACHE_ERRORS, load_recs
from metrics.accurate import getAccurateMetrics
from metrics.diversity import getDiversityMetrics
from utils.log import logger
from utils.trans import (getInteractionMatrixByDataframe, getItemDegreeByUserPosItemDict,
                         getUserItemsDictByDataframe, recommendDictToTensor)

CACHE_FILES = ("filter_rating.csv", "train_data.csv", "val_data.csv", "test_data.csv",
               "user_features.csv", "item_features.csv")


def load_preprocessed():
    """Step 1 (reference :26-56): the six preprocessed tables."""
    d = cfg.PREPROCESSING["save_path"]
    try:
        rating_df = pd.read_csv(d + "filter_rating.csv")
        train_data_df = pd.read_csv(d + "train_data.csv")
        val_data_df = pd.read_csv(d + "val_data.csv")
        test_data_df = pd.read_csv(d + "test_data.csv")
        user_features_df = pd.read_csv(d + "user_features.csv", sep="\t")
        item_features_df = pd.read_csv(d + "item_features.csv", sep="\t")
    except FileNotFoundError:
        logger.info("预处理数据读取失败，正在重新计算")
        try:
            if cfg.DATA_SET == "movielens":
                from processing.handleMovielens import prepareMovieLens as prepare
            else:
                from processing.handleDouban import prepareDouban as prepare
        except ImportError as ex:
            raise FileNotFoundError(
                f"no preprocessed data under {d} ({', '.join(CACHE_FILES)}) and no dataset "
                f"ETL package to build it (processing/ is outside this package)") from ex
        return prepare(cfg.PREPROCESSING["dataset_path_dict"], cfg.PREPROCESSING["save_path"])
    return rating_df, train_data_df, val_data_df, test_data_df, user_features_df, item_features_df


def recommend(name: str, user_num: int, item_num: int, rating_df, train_data_df, val_data_df,
              test_data_df, user_features_df, item_features_df) -> dict:
    """Step 2's dispatch (reference :67-80)."""
    if name in ("ProbS", "HeatS", "HybridS"):
        from model.SpreadMethod.recommend import recommendSpreadMethod
        return recommendSpreadMethod(user_num, item_num, train_data_df, val_data_df, name)
    if name == "LightGCN":
        from model.LightGCN.recommend import recommendLightGCN
        return recommendLightGCN(user_num, item_num, rating_df, train_data_df, val_data_df,
                                 test_data_df)
    if name == "LightGCNOpti":
        from model.LightGCNOpti.recommend import recommendLightGCNOpti
        return recommendLightGCNOpti(user_num, item_num, rating_df, train_data_df, val_data_df,
                                     test_data_df, user_features_df, item_features_df)
    if name == "SpreadLightGCN":
        from model.SpreadLightGCN.recommend import recommendSpreadLightGCN
        return recommendSpreadLightGCN(user_num, item_num, rating_df, train_data_df,
                                       val_data_df, test_data_df)
    if name == "SpreadLightGCNOpti":
        from model.SpreadLightGCNOpti.recommend import recommendSpreadLightGCNOpti
        return recommendSpreadLightGCNOpti(user_num, item_num, rating_df, train_data_df,
                                           val_data_df, test_data_df, user_features_df,
                                           item_features_df)
    raise ValueError(f"unknown model {name!r}")


def main() -> dict:
    logger.info("Step1：正在加载预处理数据")
    (rating_df, train_data_df, val_data_df, test_data_df, user_features_df,
     item_features_df) = load_preprocessed()
    user_num = len(rating_df["user_id"].unique())
    item_num = len(rating_df["item_id"].unique())
    logger.info(f"总用户数：{user_num}，总项目数：{item_num}")
    logger.info(f"训练集 ：{train_data_df.shape}")
    logger.info(f"验证集 ：{val_data_df.shape}")
    logger.info(f"测试集 ：{test_data_df.shape}")
    logger.info("预处理数据加载完毕")
    logger.info("-------------------------------------------------------")

    logger.info("Step2：正在读取推荐结果")
    name, k = cfg.MODEL["name"], cfg.RECOMMEND["k"]
    path = cfg.RECOMMEND["save_path"] + "all_user_recommend_dict_" + name + str(k) + ".npy"
    try:
        # a dict this package's recommenders saved (lgcnhs.recs.save_recs), as the reference
        # does; the name has no "_" before k, as in reference main.py:62, so (as there) only
        # LightGCNOpti's saver (no "_" either) hits this cache and the others recompute. Read
        # from the saver's pickle-free sidecar (never unpickled); any unreadable, stale or
        # foreign cache recomputes, as the reference's bare except does (main.py:61-64)
        all_user_recommend_dict = load_recs(path)
        logger.info("推荐结果读取完毕")
    except CACHE_ERRORS:
        logger.info(f"推荐结果读取失败，正在重新进行推荐，选用模型：{name}")
        all_user_recommend_dict = recommend(name, user_num, item_num, rating_df, train_data_df,
                                            val_data_df, test_data_df, user_features_df,
                                            item_features_df)
    logger.info("-------------------------------------------------------")

    logger.info("Step3：正在评估推荐结果")
    recommendations = recommendDictToTensor(all_user_recommend_dict)
    train_pos = getUserItemsDictByDataframe(train_data_df)
    val_pos = getUserItemsDictByDataframe(val_data_df)
    test_pos = getUserItemsDictByDataframe(test_data_df)
    item_degree_dict = getItemDegreeByUserPosItemDict(train_pos, val_pos)
    interaction_mat = getInteractionMatrixByDataframe(user_num, item_num,
                                                      pd.concat([train_data_df, val_data_df]))
    P, R, F1, NDCG = getAccurateMetrics(test_pos, recommendations, k)
    H, I = getDiversityMetrics(recommendations, item_degree_dict, interaction_mat, k)
    logger.info(f"[{name} Test Accurate] precision@{k}: {P}, recall@{k}: {R}, f1@{k}: {F1}, "
                f"NDCG@{k}: {NDCG}")
    logger.info(f"[{name} Test Diversity] H@{k}: {H}, I@{k}: {I}")
    return {"model": name, "k": k, "users": user_num, "items": item_num,
            "recommendations": all_user_recommend_dict, "precision": P, "recall": R,
            "f1": F1, "ndcg": NDCG, "H": H, "I": I}


if __name__ == "__main__":
    main()
