"""Sum the `cprof <slot> <cycles>` lines of tools/cprof_probe.py's output."""
import sys
NAMES = {0: "layer searches", 1: "addNeighbor append", 2: "evict: worst of M+1", 3: "evict: two removes",
         4: "replenish (total)", 5: "repl: stage rows", 6: "repl: walk ranks", 7: "repl: visited + collect",
         8: "repl: distances", 9: "repl: pops + appends", 10: "isolate sweep", 11: "mw eval (post..collect)",
         12: "mw sink loops", 13: "addNeighbor pairs (total)", 14: "repl: set path", 15: "repl: set path taken", 20: "repl: set path declined", 16: "inserts", 17: "evictions",
         18: "replenishes", 19: "replenish candidates", 21: "kernel total", 22: "search expansion batches", 23: "search candidates"}
tot = {}
for line in open(sys.argv[1]):
    p = line.split()
    if len(p) == 3 and p[0] == "cprof":
        tot[int(p[1])] = tot.get(int(p[1]), 0) + int(p[2])
ins = max(tot.get(16, 1), 1)
for s in sorted(tot):
    if tot[s]:
        print(f"{s:2d} {NAMES.get(s, '?'):28s} {tot[s]:>16d}  per insert {tot[s] / ins:12.1f}")
