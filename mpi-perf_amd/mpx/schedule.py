"""Pair schedules (Python mirror of mpxh_pairing / mpxh_round_role in
mpi-perf_amd/host/mpx_host.c).

pairing_from_groups(): the reference's group/peer rule (mpi_perf.c:447-450
Comm_split keyed by world rank; :225-233 first other-group rank with the same
group rank).

all_pairs_rounds(): circle-method 1-factorisation of K_N — N-1 rounds of N/2
disjoint pairs covering every one of the N(N-1)/2 pairs once.
Round r is exactly one reference run with ppn = N/2 on two "hosts": pair k of
the round is (G1 = logical rank k, G0 = logical rank N/2 + k).
"""
from __future__ import annotations


def pairing_from_groups(groups: list[int]) -> tuple[list[int], list[int]]:
    group_rank = []
    for r, g in enumerate(groups):
        group_rank.append(sum(1 for q in range(r) if groups[q] == g))
    peer = []
    for r, g in enumerate(groups):
        p = -1
        for i, gi in enumerate(groups):
            if gi != g and group_rank[i] == group_rank[r]:
                p = i
                break
        peer.append(p)
    return group_rank, peer


def all_pairs_rounds(n: int) -> list[list[tuple[int, int]]]:
    """Rounds of (group-1 rank, group-0 rank) pairs; n must be even (>= 2)."""
    if n < 2 or n % 2:
        raise ValueError("all-pairs rounds need an even number of ranks >= 2")
    order = list(range(n))
    rounds = []
    for _ in range(n - 1):
        rounds.append([(order[k], order[n - 1 - k]) for k in range(n // 2)])
        order = [order[0], order[-1]] + order[1:-1]
    return rounds


def round_role(rounds: list[list[tuple[int, int]]], r: int, rank: int) -> tuple[int, int]:
    """(group, peer) of `rank` in round r."""
    for a, b in rounds[r]:
        if rank == a:
            return 1, b
        if rank == b:
            return 0, a
    raise ValueError(f"rank {rank} not scheduled in round {r}")
