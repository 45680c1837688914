"""LGCNHS recommendation with the reference's interface
(reference model/SpreadLightGCNOpti/recommend.py:18-79), fused on the GPU as
model.SpreadLightGCN.recommend.spread_lightgcn_topk."""
import pandas as pd

from const import cfg
from model.SpreadLightGCN.recommend import (_save, _to_dict, recommendForAllUser,  # noqa: F401
                                            spread_lightgcn_topk)


def recommendSpreadLightGCNOpti(user_num: int, item_num: int, rating_df: pd.DataFrame,
                                train_data_df: pd.DataFrame, val_data_df: pd.DataFrame,
                                test_data_df: pd.DataFrame, user_features_df: pd.DataFrame,
                                item_features_df: pd.DataFrame) -> dict:
    from model.SpreadLightGCNOpti.model import getLightGCNOptiModel
    k = cfg.RECOMMEND["k"]
    model = getLightGCNOptiModel(user_num, item_num, rating_df, train_data_df, val_data_df,
                                 test_data_df, user_features_df, item_features_df, k)[0]
    _, idx = spread_lightgcn_topk(model, user_num, item_num, train_data_df, val_data_df,
                                  cfg.MODEL["HyperParameter"]["lambda"], k)
    recs = _to_dict(idx, user_num)
    _save(recs)
    return recs
