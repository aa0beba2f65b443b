"""Per-kernel floor of dependent launches on one stream: N back-to-back tiny kernels (our fill_f32 on a
few elements), eager and replayed from a hipGraph; and the same with a 2048-block grid.  Answers what a
dispatch costs when its work is negligible (ResNet-18 CIFAR: ~165 dependent kernels per step)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from deeplearning_mpi_amd._ext import native
    C = native()
    small = torch.empty(64, device="cuda")
    big = torch.empty(2048 * 256, device="cuda")
    n = 2000
    out = {}
    for name, buf in (("tiny_1block", small), ("tiny_2048blocks", big)):
        f = lambda: C.fill_(buf, 0.0)
        for _ in range(50):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            f()
        e.record()
        torch.cuda.synchronize()
        out[name + "_eager_us"] = round(s.elapsed_time(e) / n * 1e3, 2)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            f()
            with torch.cuda.graph(g, stream=st):
                for _ in range(200):
                    f()
        torch.cuda.current_stream().wait_stream(st)
        g.replay()
        torch.cuda.synchronize()
        s.record()
        for _ in range(n // 200):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        out[name + "_graph_us"] = round(s.elapsed_time(e) / n * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
