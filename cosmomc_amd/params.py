"""Parameter blocking for the BlockedProposer: a restatement of
TBaseParameters_SetFastSlowParams (source/BaseParameters.f90:302-433).

The reference sorts the varying parameters into speed types -- slow, semi-slow,
semi-fast, fast -- and, with block_fast_likelihood_params (default .true.,
BaseParameters.f90:34), cuts the fast parameters into one block per likelihood
"so not randomly mix them and hence don't all need to be recomputed"
(:360-362).  The blocks feed BlockedProposer%Init with slow_block_max =
slow_tp_max = tp_semislow (MCMC.f90:261), i.e. BatchedMCMC(blocks=...,
slow_block_max=2).  With the per-likelihood change mask (calclike.f90:374-386,
mh_kernel) a step that moves one likelihood's block re-evaluates only that
likelihood.

The block boundaries follow the reference exactly, including where it puts
them: the break for a likelihood is recorded at the used index j of that
likelihood's first fast parameter, and a block runs up to and including its
break (:406-418), so every block after the first starts one parameter into
its likelihood's set and the previous block ends with that parameter.
"""
from __future__ import annotations

from dataclasses import dataclass, field

TP_UNUSED, TP_SLOW, TP_SEMISLOW, TP_SEMIFAST, TP_FAST = 0, 1, 2, 3, 4   # BaseParameters.f90:11
SLOW_TP_MAX = TP_SEMISLOW                                              # :13


@dataclass
class FastSlowBlocks:
    param_blocks: list                    # [tp_semifast + num_breaks] lists of used indices (1-based)
    slow_block_max: int = SLOW_TP_MAX
    num_fast: int = 0
    num_slow: int = 0
    num_semi_slow: int = 0
    num_semi_fast: int = 0
    breaks: list = field(default_factory=list)
    param_type: list = field(default_factory=list)   # per parameter 1..num_params (index 0 unused)


def set_fast_slow_params(num_params: int, varying, likes, num_theory_params: int, use_fast_slow: bool = True,
                         fast_parameters=None, fast_param_index: int | None = None, index_semislow: int = -1,
                         block_semi_fast: bool = True, block_fast_likelihood_params: bool = True) -> FastSlowBlocks:
    """varying: num_params booleans (BaseParams%varying); likes: the sorted
    likelihood list after LikelihoodList.add_nuisance_parameters (each with
    new_param_block_start / new_params, GeneralTypes.f90:638-641, and speed);
    num_theory_params: index_data - 1 (GeneralTypes.f90:185).
    fast_parameters: 1-based parameter indices (the 'fast_parameters' ini
    names, already mapped), else every parameter from fast_param_index
    (default max(index_data, first_fast_param), :323) up is fast."""
    index_data = num_theory_params + 1
    params_used = [i for i in range(1, num_params + 1) if varying[i - 1]]
    n_used = len(params_used)
    if use_fast_slow:
        if fast_parameters is not None:
            fast = list(fast_parameters)
        else:
            first_fast = 0
            for like in likes:                       # TLikelihoodList%first_fast_param (:650-651)
                if first_fast == 0 and like.speed >= 0 and like.new_params > 0:
                    first_fast = like.new_param_block_start
            fpi = max(index_data, first_fast) if fast_param_index is None else fast_param_index
            fast = list(range(fpi, num_params + 1))
    else:
        fast = []
        block_semi_fast = False
        block_fast_likelihood_params = False
    ptype = [TP_UNUSED] * (num_params + 1)
    for i in range(1, num_params + 1):                # :341-356
        if not varying[i - 1]:
            continue
        if use_fast_slow and i in fast:
            ptype[i] = TP_FAST if (i >= index_data or not block_semi_fast) else TP_SEMIFAST
        elif use_fast_slow and index_semislow >= 0 and i >= index_semislow and block_semi_fast:
            ptype[i] = TP_SEMISLOW
        else:
            ptype[i] = TP_SLOW
    breaks = []
    if block_fast_likelihood_params:                  # :360-378
        first = True
        for like in likes:
            for j in range(1, n_used):                # j = 1 .. num_params_used - 1
                p = params_used[j - 1]
                if ptype[p] == TP_FAST and like.new_param_block_start <= p < like.new_param_block_start + like.new_params:
                    if first:
                        first = False
                    else:
                        breaks.append(j)
                    break
    breaks.append(n_used)
    breaks = _order_indices(breaks)
    out = FastSlowBlocks(param_blocks=[], breaks=list(breaks), param_type=ptype)
    for speed in (TP_SLOW, TP_SEMISLOW, TP_SEMIFAST):  # :391-405
        blk = []
        for i in range(1, n_used + 1):
            if ptype[params_used[i - 1]] == speed:
                if speed <= SLOW_TP_MAX:
                    out.num_slow += 1
                else:
                    out.num_fast += 1
                blk.append(i)
        out.param_blocks.append(blk)
    ix = 1
    for j in breaks:                                  # :406-418: ix .. j inclusive
        blk = [i for i in range(ix, j + 1) if ptype[params_used[i - 1]] == TP_FAST]
        out.num_fast += len(blk)
        out.param_blocks.append(blk)
        ix = j + 1
    out.num_semi_slow = len(out.param_blocks[TP_SEMISLOW - 1])
    out.num_semi_fast = len(out.param_blocks[TP_SEMIFAST - 1])
    return out


def _order_indices(arr):
    """orderIndices (BaseParameters.f90:285-299): the breaks in ascending order
    (a selection sort; duplicates kept)."""
    return sorted(arr)
