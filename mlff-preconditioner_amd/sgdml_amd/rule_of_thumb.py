"""Rule-of-thumb preconditioner size used by the reference's solver entry point
(src/train_models.py:93-97 -> src/tools/plot_data.py:677-734, 1254-1258)."""
from __future__ import annotations

import math

# plot_data.get_params(old=False): dataset -> (slope m, k_unity k_min)
_PARAMS = {
    "default": (1.0, 100), "ethanol": (0.87, 10), "uracil": (1.07, 32),
    "C6H5CH3": (1.01, 44), "toluene": (1.01, 44), "aspirin": (1.14, 236),
    "azobenzene_new": (1.02, 62), "azobenzene": (1.02, 62),
    "aims_catcher": (1.02, 316), "catcher": (1.02, 316),
    "larger_aims_nanotube": (0.73, 89), "nanotube": (0.73, 89),
}


def get_params(dataset_name: str, old: bool = False):
    """Returns (slope, k_unity, prefactor) like plot_data.get_params."""
    if old:
        raise NotImplementedError("only the current (old=False) rule-of-thumb table is used by train_models.py")
    if dataset_name not in _PARAMS:
        raise NotImplementedError(f"dataset_name = {dataset_name} is not specified. ")
    m, k = _PARAMS[dataset_name]
    return m, k, 1


def rule_of_thumb(n, k_min, m):
    """k = floor((k_min^m * m * n^2 / 2)^(1/(2+m))) for integer n (plot_data.py:1254-1258)."""
    res = (k_min ** m * m * n ** 2 / 2) ** (1 / (2 + m))
    if isinstance(n, int):
        res = int(math.floor(res))
    return res


def break_percentage(n: int, dataset_name: str) -> float:
    """preconditioner_strength = k_RoT / n (src/train_models.py:95-97)."""
    m, k_min, _ = get_params(dataset_name)
    return int(rule_of_thumb(n=int(n), k_min=k_min, m=m)) / n
