"""CLI mirror of provided/main.py:14-35.

    python -m rtx.main --infile S.json --outfile out.png [--subimage k --tasks N]

Full render: rot90 + truncating uint8 conversion + PNG (main.py:29-34; the viewer call
`im.show()` at :35 is not reproduced). Strip render: numpy.save of the (strip_w, H, 3)
float64 strip (main.py:26-28), for rtx.glue. Extensions: --resolution W H and --spp AA [DOF]
edit the scene like the bench configs; --distributed renders row blocks on every rank
of a torch.distributed job and gathers the frame to rank 0 (render.nu's role).
"""
import argparse
import json
import os

import numpy


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--infile", type=str, help="Name of json file that will define the scene")
    p.add_argument("--outfile", type=str, default="out.png", help="Name of png that will contain the render")
    p.add_argument("--subimage", type=int, required=False)
    p.add_argument("--tasks", type=int, required=False)
    p.add_argument("--resolution", type=int, nargs=2, default=None)
    p.add_argument("--spp", type=int, nargs="+", default=None, help="AA samples [DOF samples]")
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--quiet", action="store_true")
    return p.parse_args(argv)


def _scene(args):
    from .scene_parser import load_scene
    if args.resolution is None and args.spp is None:
        return load_scene(args.infile, verbose=not args.quiet)
    with open(args.infile) as f:
        data = json.load(f)
    if args.resolution is not None:
        data["resolution"] = list(args.resolution)
    if args.spp is not None:
        data.setdefault("AA", {"jitter": False, "samples": 1})["samples"] = args.spp[0]
        if len(args.spp) > 1:
            data.setdefault("DOF", {"focal_length": 1, "aperture": 0, "samples": 1})["samples"] = args.spp[1]
    data["__base_dir__"] = os.path.dirname(os.path.abspath(args.infile))
    return load_scene(data, verbose=not args.quiet)


def main(argv=None):
    args = parse(argv)
    import torch
    from PIL import Image
    if args.distributed:
        import torch.distributed as dist
        from .distributed import render_frame
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        rank, world = dist.get_rank(), dist.get_world_size()
        sc = _scene(args)
        frame = render_frame(sc, rank, world, dtype=torch.uint8)
        if rank == 0:
            Image.fromarray(frame.cpu().numpy()).save(args.outfile)
        dist.destroy_process_group()
        return
    full_scene = _scene(args)
    if args.subimage is not None and args.tasks is not None:
        image = full_scene.render(args.subimage, args.tasks)
        numpy.save(args.outfile, image)
    else:
        rgb = full_scene.render_rgb8()  # == (rot90(render()) * 255).astype(uint8), on the device
        Image.fromarray(rgb).save(args.outfile)


if __name__ == "__main__":
    main()
