"""The chain kernel's run replay (k_chain in canu_amd/csrc/ovl_seed.hip) is
exact: a model of Add_Match (overlapInCore-Find_Overlaps.C:79: extend the head node when the
occurrence is the next window on its diagonal, else walk the list -- move-to-front, the
consistency rule -- else push a new node) applied entry by entry gives the same node lists and
flags as applying an entry and then its whole run at once, where a run entry follows the
previous entry of the target's list by one window on the same diagonal and both are their
windows' only occurrence.  Random match sequences with repeats, diagonal shifts and stray
hits."""
import random

K = 22


def add_match(s, p, o):
    nodes = s["nodes"]                      # list order, head first: [Offset, Len, Start]
    new_diag = p - o
    diag = expected = checked = 0
    if nodes:
        hd = nodes[0]
        expected, diag = hd[2] + hd[1] - K + 1, hd[0] - hd[2]
        if expected == o and new_diag == diag:
            hd[1] += 1
            return
        if expected >= o:
            mtf, checked = expected == o, 1
            for idx in range(1, len(nodes)):
                nd = nodes[idx]
                expected, diag = nd[2] + nd[1] - K + 1, nd[0] - nd[2]
                if expected < o:
                    break
                if expected == o:
                    if new_diag == diag:
                        nd[1] += 1
                        if mtf:
                            nodes.insert(0, nodes.pop(idx))
                        return
                    mtf = True
                checked += 1
        if checked > 0 or abs(diag - new_diag) > 3 or o < expected + K - 2:
            s["consistent"] = 0
    nodes.insert(0, [p, K, o])


def replay_plain(entries):
    s = {"nodes": [], "consistent": 1}
    for o, p in entries:
        add_match(s, p, o)
    return s


def replay_runs(entries):
    n = len(entries)
    cont = [False] * n
    for i in range(1, n):
        (o, p), (ow, pw) = entries[i], entries[i - 1]
        cont[i] = (ow + 1 == o and p - o == pw - ow and
                   (i + 1 >= n or entries[i + 1][0] != o) and
                   (i < 2 or entries[i - 2][0] != ow))
    s = {"nodes": [], "consistent": 1}
    i = 0
    while i < n:
        run = 0
        while i + 1 + run < n and cont[i + 1 + run]:
            run += 1
        o, p = entries[i]
        add_match(s, p, o)
        i += 1
        hd = s["nodes"][0] if s["nodes"] else None
        if run and hd and hd[2] + hd[1] - K == o and hd[0] - hd[2] == p - o:
            hd[1] += run
            i += run
    return s


def test_run_replay_equals_entry_replay():
    rng = random.Random(1)
    for _ in range(3000):
        entries, o, diag = [], 0, rng.randint(-50, 50)
        for _ in range(rng.randint(1, 200)):
            o += 1
            r = rng.random()
            if r < 0.8:
                entries.append((o, o + diag))
            elif r < 0.85:
                diag += rng.choice([-2, -1, 1, 2])
                entries.append((o, o + diag))
            elif r < 0.9:                     # a repeat: two occurrences in one window
                entries.append((o, o + diag))
                entries.append((o, o + diag + rng.randint(-30, 30)))
            elif r < 0.95:                    # a stray hit
                entries.append((o, o + rng.randint(-100, 100)))
        assert replay_runs(entries) == replay_plain(entries)
