"""What HIP leaves behind after an invalidated hipGraph capture (utils/graphs.py fallback design).

Observed on ROCm 7.2 / gfx950: hipStreamEndCapture does not close the invalidated capture; the
capture stream AND the capturing thread's legacy default stream keep reporting capture mode and
refuse every launch from that thread.  A capture begun on a helper thread leaves the main thread
usable (only the abandoned capture stream stays stuck)."""
import os
import sys
import threading

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch  # noqa: E402

from deeplearning_mpi_amd._ext import native  # noqa: E402

C = native()
x = torch.ones(4, device="cuda")


def failing_capture(stream):
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            y = x * 2
            float(y.sum())
    except Exception as e:   # noqa: BLE001
        print("capture raised:", str(e).splitlines()[0])


def probe(tag):
    for name, fn in [("torch fill", lambda: x.fill_(3)), ("dlmpi fill", lambda: C.fill_(x, 1.0))]:
        try:
            fn()
            torch.cuda.synchronize()
            print(tag, name, "ok")
        except Exception as e:   # noqa: BLE001
            print(tag, name, "FAILED:", str(e).splitlines()[0])
            C.clear_hip_error()


mode = sys.argv[1] if len(sys.argv) > 1 else "thread"
s = torch.cuda.ExternalStream(C.create_stream())
if mode == "same":
    failing_capture(s)
else:
    t = threading.Thread(target=failing_capture, args=(s,))
    t.start()
    t.join()
print("capture stream still capturing:", C.stream_capturing(s.cuda_stream))
C.clear_hip_error()
probe(mode)
