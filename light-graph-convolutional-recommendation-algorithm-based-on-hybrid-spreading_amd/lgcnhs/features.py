"""Feature-table parsing shared by the Opti models (reference
model/LightGCNOpti/recommend.py:150-163, model/SpreadLightGCNOpti/model.py:59-76)."""
import ast

import numpy as np
import pandas as pd
import torch


def features_tensor(df: pd.DataFrame, id_col: str, feat_col: str) -> torch.Tensor:
    rows = df.sort_values(by=id_col)[feat_col].apply(
        lambda r: ast.literal_eval(r) if not isinstance(r, list) else r).tolist()
    return torch.from_numpy(np.array(rows)).float()
