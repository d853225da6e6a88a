"""Worker of tests/test_watchdog_cpu.py: a gloo world of two ranks under SetupWatchdog.
mode "withhold": rank 1 never enters the barrier rank 0 waits in (it stalls in a step of its
own); both ranks must exit with the watchdog's status within its bound.  mode "ok": both enter
the barrier and finish normally."""
import datetime
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch.distributed as dist  # noqa: E402

from DistGNN.dist.watchdog import SetupWatchdog  # noqa: E402


def main(mode, bound):
    rank = int(os.environ["RANK"])
    wd = SetupWatchdog(bound, rank=rank, what="test setup", exit_code=3)
    wd.step("init_process_group")
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=120))
    if mode == "withhold" and rank == 1:
        wd.step("rank 1 work before the barrier")
        time.sleep(120)  # withholds the collective
    wd.step("barrier")
    dist.barrier()
    wd.done()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]))
