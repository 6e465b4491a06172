"""Seeding state-machine load model from the emulator's per-seed trip counts (dev tool).

  build/emu/emu_prof <index> <reads.fq> > prof.txt   (EMU_WAVE=1; lines "R i L |F t,m ... |S t,m ...")
  python tools/seed_prof.py prof*.txt

For every read and phase (F = fast, S = slow) it models the wave's trip count on the GPU:
  ideal    sum of trips / 64 lanes
  greedy   seeds handed out in order to the first free lane, no map barrier
  barrier  the current state machine: a lane that reached MAP waits until every active lane
           has (DSB_SM_MAP_BATCH = 64), one map per lane per map trip
and prints the distribution over reads; the slow phase's kernel time is set by its slowest read.
"""
import heapq
import sys


def parse(paths):
    for p in paths:
        for line in open(p):
            if not line.startswith("R "):
                continue
            head, rest = line.split("|F")
            fpart, spart = rest.split("|S")
            _, i, L = head.split()[:3]
            f = [tuple(map(int, x.split(","))) for x in fpart.split()]
            s = [tuple(map(int, x.split(","))) for x in spart.split()]
            yield int(i), int(L), f, s


def greedy(seeds, lanes=64):
    h = [0] * min(lanes, len(seeds))
    heapq.heapify(h)
    for t, _ in seeds:
        heapq.heappush(h, heapq.heappop(h) + t)
    return max(h) if h else 0


def barrier(seeds, lanes=64, map_cost=1, batch=64):
    """slow seeds: search trips, then `maps` map steps; a map step runs only when every active
    lane is waiting to map (or >= batch lanes wait)"""
    q = list(seeds)
    lane = []  # [search_left, maps_left]
    nxt = 0
    for _ in range(min(lanes, len(q))):
        t, m = q[nxt]
        lane.append([max(0, t - m), m])
        nxt += 1
    time = 0
    while lane:
        waiting = [l for l in lane if l[0] == 0 and l[1] > 0]
        searching = [l for l in lane if l[0] > 0]
        if waiting and (not searching or len(waiting) >= batch):
            time += map_cost
            for l in waiting:
                l[1] -= 1
        else:
            # advance searching lanes to the next event (one of them reaching MAP)
            step = min(l[0] for l in searching)
            time += step
            for l in searching:
                l[0] -= step
        done = [l for l in lane if l[0] == 0 and l[1] == 0]
        for l in done:
            lane.remove(l)
            if nxt < len(q):
                t, m = q[nxt]
                nxt += 1
                lane.append([max(0, t - m), m])
    return time


def main():
    rows = list(parse(sys.argv[1:]))
    slow = [(i, L, s) for i, L, f, s in rows if s]
    print(f"reads {len(rows)}  with slow seeding {len(slow)}")
    res = []
    for i, L, s in slow:
        tot = sum(t for t, _ in s)
        res.append((barrier(s, map_cost=4), greedy(s), tot / 64, tot, len(s), L, i, max(t for t, _ in s)))
    res.sort(reverse=True)
    print("slow reads, slowest first: barrier(map=4) greedy ideal sum n_seeds L read max_seed")
    for r in res[:25]:
        print("  %7d %7d %8.1f %8d %5d %6d %6d %5d" % r)
    import statistics
    for k, nm in ((0, "barrier"), (1, "greedy"), (2, "ideal")):
        v = [r[k] for r in res]
        print(f"{nm:8s} max {max(v):9.0f} p99 {sorted(v)[int(0.99 * len(v))]:9.0f} mean {statistics.mean(v):9.1f} sum {sum(v):11.0f}")
    fast = []
    for i, L, f, s in rows:
        if f:
            tot = sum(t for t, _ in f)
            fast.append((greedy(f), tot / 64, tot, len(f), L))
    v0 = [r[0] for r in fast]
    v2 = [r[1] for r in fast]
    print(f"fast: reads {len(fast)} greedy sum {sum(v0):.0f} max {max(v0)}  ideal sum {sum(v2):.0f}")


if __name__ == "__main__":
    main()
