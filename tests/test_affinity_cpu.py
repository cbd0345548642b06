"""CPU: per-rank host CPU groups of the multi-GPU bench (rabbitsalign_amd.shard.rank_cpu_groups):
ranks spread over NUMA nodes in order, SMT siblings stay together, no two ranks share a core."""
from rabbitsalign_amd import shard


def _two_socket(cores_per_node=64, smt=True):
    n0 = list(range(0, cores_per_node)) + (list(range(2 * cores_per_node, 3 * cores_per_node)) if smt else [])
    n1 = list(range(cores_per_node, 2 * cores_per_node)) + (list(range(3 * cores_per_node, 4 * cores_per_node)) if smt else [])
    sib = {}
    for c in range(2 * cores_per_node):
        pair = (c, c + 2 * cores_per_node) if smt else (c,)
        for x in pair:
            sib[x] = pair
    return [n0, n1], sib


def test_eight_ranks_two_sockets():
    nodes, sib = _two_socket()
    g = shard.rank_cpu_groups(nodes, sib, 8)
    assert [len(x) for x in g] == [32] * 8
    allc = [c for x in g for c in x]
    assert len(allc) == len(set(allc)) == 256                     # disjoint, complete
    for r in range(4):
        assert all(c in nodes[0] for c in g[r])
        assert all(c in nodes[1] for c in g[r + 4])
    for x in g:                                                    # siblings together
        for c in x:
            assert all(s in x for s in sib[c])


def test_uneven_and_small():
    nodes, sib = _two_socket(cores_per_node=6, smt=False)
    g = shard.rank_cpu_groups(nodes, sib, 3)                       # ranks 0,1 -> node 0; rank 2 -> node 1
    assert sorted(g[0] + g[1]) == nodes[0] and g[2] == nodes[1]
    g = shard.rank_cpu_groups([[0, 1]], {0: (0,), 1: (1,)}, 4)     # more ranks than cores: share
    assert all(x for x in g)
    g = shard.rank_cpu_groups([[], [4, 5, 6, 7]], {c: (c,) for c in range(4, 8)}, 2)
    assert g == [[4, 5], [6, 7]]


def test_parse_cpulist():
    assert shard._parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
