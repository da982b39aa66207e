"""Executable model of the selection algorithm the HIP ball-query / 3-NN kernels run.

PyTorch-CPU `topk(k, largest=False)` (the reference's `group` and
`interpolate`, models/utils/common.py:61,114) builds (value, index) pairs in
index order and runs libstdc++ `partial_sort` when k*64 <= n, else
`nth_element` (+ sort of the first k-1).  Which *inf* entries pad an
underfull ball, and which of several equal distances survive, are decided by
those algorithms, so the HIP kernels emulate them:

* `heap_select`  -- partial_sort's heap select (make_heap / adjust_heap /
  push_heap), run by the kernel as wave-uniform scalar code over a heap kept in
  lanes.
* `introselect`  -- nth_element with median-of-3 pivots and Hoare partition,
  where the kernel runs each partition WAVE-PARALLEL.  `partition_parallel`
  is the closed form the kernel evaluates (left/right stop lists, crossing
  rank i*) and is checked here against the literal serial partition.

Only `tests/` use this module.
"""
from __future__ import annotations


def _lt(a, b):
    return a[0] < b[0]


# ---------------------------------------------------------------- heap select
def adjust_heap(h, hole, length, value):
    top = hole
    second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if _lt(h[second], h[second - 1]):
            second -= 1
        h[hole] = h[second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        h[hole] = h[second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and _lt(h[parent], value):
        h[hole] = h[parent]
        hole = parent
        parent = (hole - 1) // 2
    h[hole] = value


def make_heap(h, first, last):
    length = last - first
    if length < 2:
        return
    sub = h[first:last]
    parent = (length - 2) // 2
    while True:
        adjust_heap(sub, parent, length, sub[parent])
        if parent == 0:
            break
        parent -= 1
    h[first:last] = sub


def heap_select(q, first, middle, last):
    """libstdc++ __heap_select on q[first:last] keeping q[first:middle]."""
    make_heap(q, first, middle)
    sub = q[first:middle]
    for i in range(middle, last):
        if _lt(q[i], sub[0]):
            v = q[i]
            q[i] = sub[0]
            adjust_heap(sub, 0, middle - first, v)
    q[first:middle] = sub


# ---------------------------------------------------------------- introselect
def move_median_to_first(q, result, a, b, c):
    if _lt(q[a], q[b]):
        if _lt(q[b], q[c]):
            q[result], q[b] = q[b], q[result]
        elif _lt(q[a], q[c]):
            q[result], q[c] = q[c], q[result]
        else:
            q[result], q[a] = q[a], q[result]
    elif _lt(q[a], q[c]):
        q[result], q[a] = q[a], q[result]
    elif _lt(q[b], q[c]):
        q[result], q[c] = q[c], q[result]
    else:
        q[result], q[b] = q[b], q[result]


def partition_serial(q, first, last, pivot):
    while True:
        while _lt(q[first], q[pivot]):
            first += 1
        last -= 1
        while _lt(q[pivot], q[last]):
            last -= 1
        if not first < last:
            return first
        q[first], q[last] = q[last], q[first]
        first += 1


def partition_parallel(q, lo, hi, pv):
    """Closed form of partition_serial(q, lo, hi, pivot) used by the kernel.

    Lo = ascending positions with !(q < pv)  (left-scan stops),
    Ro = descending positions with !(pv < q) (right-scan stops);
    i* = #{i : Lo[i] < Ro[i]}; swaps are (Lo[i], Ro[i]) for i < i*;
    cut = Lo[i*] if it exists and (i* == 0 or Lo[i*] < Ro[i*-1]) else Ro[i*-1].
    """
    Lo = [p for p in range(lo, hi) if not q[p][0] < pv]
    Ro = [p for p in range(hi - 1, lo - 1, -1) if not pv < q[p][0]]
    # kernel form: for left stop p of rank i, Lo[i] < Ro[i]  <=>  #right stops > p  >= i+1
    istar = 0
    for i, p in enumerate(Lo):
        n_right_above = sum(1 for r in Ro if r > p)
        if n_right_above >= i + 1:
            istar = i + 1
    for i in range(istar):
        a, b = Lo[i], Ro[i]
        q[a], q[b] = q[b], q[a]
    if istar < len(Lo) and (istar == 0 or Lo[istar] < Ro[istar - 1]):
        return Lo[istar]
    return Ro[istar - 1]


def insertion_sort(q, first, last):
    for i in range(first + 1, last):
        v = q[i]
        if _lt(v, q[first]):
            q[first + 1:i + 1] = q[first:i]
            q[first] = v
        else:
            j = i
            while _lt(v, q[j - 1]):
                q[j] = q[j - 1]
                j -= 1
            q[j] = v


def introselect(q, nth, parallel=False):
    first, last = 0, len(q)
    if first == last or nth == last:
        return
    depth = 2 * (len(q).bit_length() - 1)
    while last - first > 3:
        if depth == 0:
            heap_select(q, first, nth + 1, last)
            q[first], q[nth] = q[nth], q[first]
            return
        depth -= 1
        mid = first + (last - first) // 2
        move_median_to_first(q, first, first + 1, mid, last - 1)
        if parallel:
            cut = partition_parallel(q, first + 1, last, q[first][0])
        else:
            cut = partition_serial(q, first + 1, last, first)
        if cut <= nth:
            first = cut
        else:
            last = cut
    insertion_sort(q, first, last)


def topk_smallest_set(values, k, parallel=False):
    """Index set CPU torch.topk(values, k, largest=False) returns."""
    n = len(values)
    q = [(float(v), i) for i, v in enumerate(values)]
    if k * 64 <= n:
        heap_select(q, 0, k, n)
    else:
        introselect(q, k - 1, parallel)
    return sorted(i for _, i in q[:k])
