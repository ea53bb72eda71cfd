"""Stand-in for bench.py under bench.launch_ranks (tests/test_launcher.py): forms the gloo group the
launcher's environment describes, all-reduces the ranks, and prints one JSON line on rank 0;
``--fail-rank R`` makes rank R exit 3 before the rendezvous."""
import json
import os
import sys

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if "--fail-rank" in sys.argv and int(sys.argv[sys.argv.index("--fail-rank") + 1]) == rank:
    sys.exit(3)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
t = torch.tensor([rank + 1])
dist.all_reduce(t)
if rank == 0:
    print(json.dumps({"world": world, "rank_sum": int(t.item()), "master_addr": os.environ.get("MASTER_ADDR"),
                      "local_ranks": world, "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
