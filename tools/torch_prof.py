"""Op-level attribution of the bench step's GPU time (torch.profiler): which
aten / custom ops launch which kernels.  python tools/torch_prof.py [bench args]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    from apex_example_amd.utils.dist import init_distributed

    rank, world, device = init_distributed()
    torch.manual_seed(0)
    w = bench.build_resnet(args, device, world) if args.model.startswith("resnet") else (
        bench.build_bert(args, device, world) if args.model == "bert_large"
        else bench.build_gpt2(args, device, world))
    for _ in range(5):
        w.step(w.batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        for _ in range(2):
            w.step(w.batch)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_cuda_time_total", row_limit=int(os.environ.get("TORCH_PROF_ROWS", "60")), max_name_column_width=60,
                   max_shapes_column_width=90))


if __name__ == "__main__":
    main()
