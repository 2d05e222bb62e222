"""Recall evaluation on the GPU searcher (reference: backend/utils/eval_utils.py:85-147).

Deviation D-click-index: the reference's get_click_index (:85-99) builds its "miss" mask from
`np.ones_like(rec_id[:, 0]) == label_id` (compares the label with 1, not with the first recommendation),
so a hit at position 0 of a label other than 1 is scored as a miss and a miss of label 1 as a hit at 0.
The build returns the intended value: the first position of the label in the list, or 1e14 when absent.
The metric formulas (:138-144) are kept verbatim.
"""
from __future__ import annotations

import time
from typing import List, Tuple

import numpy as np

MISS = int(1e14)


def get_click_index(rec_id: np.ndarray, label_id: np.ndarray) -> np.ndarray:
    assert rec_id.shape[0] == label_id.shape[0], "Sample nums does not match!"
    hit = rec_id == label_id[:, None]
    pos = hit.argmax(axis=1).astype(np.int64)
    pos[~hit.any(axis=1)] = MISS
    return pos


def batch_get_click_ids(searcher, targets, labels, batch_size, k):
    start = time.time()
    out = []
    for i in range(0, len(targets), batch_size):
        rec_ids = searcher.search(targets[i:i + batch_size], k)
        out.append(get_click_index(rec_ids[0], np.asarray(labels[i:i + batch_size])))
    click_ids = np.hstack(out) if out else np.zeros(0, np.int64)
    print(f"Batch search recall cost: {time.time() - start}")
    return click_ids


def batch_compute_recall_score(searcher, targets: np.ndarray, labels: np.ndarray, topk_list: List[int],
                               weights: np.ndarray, batch_size: int) -> Tuple[List[float], List[float], List[float]]:
    """hit@K, mrr, ndcg@K (eval_utils.py:120-147)."""
    click_ids = batch_get_click_ids(searcher, targets, labels, batch_size, max(topk_list))
    hit, mrr, ndcg = [], [], []
    for k in topk_list:
        info = (click_ids < k).astype(int)
        dcgs = 1 / np.log2(click_ids + 2) * info
        i_dcgs = 1 / np.log2(info + 2) * info + 1e-12
        hit.append((info * weights).sum() / (weights.sum() + 1e-12))
        mrr.append(((1 / (click_ids + 1)) * weights).sum() / (weights.sum() + 1e-12))
        ndcg.append(((dcgs / i_dcgs) * weights).sum() / (weights.sum() + 1e-12))
    return hit, mrr, ndcg
