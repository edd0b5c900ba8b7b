"""The input-handler path alone (bench.py's via_input_handler: 1e8 config-4 events as host columns through
sm_input_send_columns to a counting StreamCallback), for a rocprofv3 kernel / copy trace of its chunk pipeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sym, price, vol, tsa, ts = bench.gen_stock(0, n, 1_000_000, 10000, dev, bench.seed_for(4))
    from siddhi_amd.testing import ProductApp
    app = ProductApp(bench.APP)
    app.set_collect(False)
    app.process_device_batch("StockStream", ts, [sym, price, price, price])
    expect = app.device_matches("q")[1]
    app.close()
    r = bench.via_input_handler([sym, price, vol, tsa, ts], n, expect)
    print({k: r[k] for k in ("value", "ms", "host_ms_last_run")})


if __name__ == "__main__":
    main()
