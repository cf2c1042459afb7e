"""``python -m kdl.cli <command>``: TF-free model tooling.

  show <saved_model_dir>                     saved_model_cli-style signature dump (guide.md:202)
  convert-savedmodel <saved_model_dir> <out> SavedModel -> kdl_params.safetensors (BN folded into
                                             the conv kernels, kernels bf16: kdl.ingest.fold;
                                             --keep-bn: the Keras fp32 variables as they are)
                                             + kdl_model.json (head, signatures)
  make-synthetic <repo>/<version> [--seed] [--model xception|resnet50|vit_b16|efficientnet_b7]
                                             random-init weights of the exact architecture (Xception:
                                             a SavedModel; other families: torchvision-layout safetensors)
  serve [server flags...]                    same as python -m kdl.serving
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="kdl")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("show")
    s.add_argument("dir")
    c = sub.add_parser("convert-savedmodel")
    c.add_argument("src")
    c.add_argument("dst")
    c.add_argument("--keep-bn", action="store_true", help="write the unfolded fp32 variables")
    m = sub.add_parser("make-synthetic")
    m.add_argument("dst")
    m.add_argument("--seed", type=int, default=0)
    m.add_argument("--residual-offset", type=int, default=0)
    m.add_argument("--model", default="xception")
    sv = sub.add_parser("serve")
    sv.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.cmd == "show":
        from .ingest.savedmodel import SavedModelDir
        print(SavedModelDir(a.dir).show())
    elif a.cmd == "convert-savedmodel":
        from safetensors.torch import save_file

        from .ingest.keras_map import to_xception_params
        from .ingest.savedmodel import SavedModelDir
        sm = SavedModelDir(a.src)
        params, head = to_xception_params(sm.variables())
        out = Path(a.dst)
        out.mkdir(parents=True, exist_ok=True)
        if not a.keep_bn:
            from .ingest.fold import fold_xception
            params = fold_xception(params)
        save_file({k: v.contiguous() for k, v in params.items()}, str(out / "kdl_params.safetensors"))
        sigs = {n: {"input_key": next(iter(sg.inputs)), "input_dtype": next(iter(sg.inputs.values())).dtype,
                    "output_key": next(iter(sg.outputs))} for n, sg in sm.signatures.items() if sg.inputs}
        meta = {"head": {"hidden": head.hidden, "out": head.out, "hidden_units": head.hidden_units,
                         "classes": head.classes}, "signatures": sigs, "source": str(a.src),
                "bn_folded": not a.keep_bn}
        (out / "kdl_model.json").write_text(json.dumps(meta, indent=1))
        print(f"wrote {out}/kdl_params.safetensors ({len(params)} tensors)")
    elif a.cmd == "make-synthetic":
        if a.model != "xception":
            from safetensors.torch import save_file

            from .engine import registry
            info = registry.get(a.model)
            dst = Path(a.dst)
            dst.mkdir(parents=True, exist_ok=True)
            params = {k: v.contiguous() for k, v in info.init_params(a.seed).items()}
            save_file(params, str(dst / "kdl_params.safetensors"))
            (dst / "kdl_model.json").write_text(json.dumps({"family": a.model}))
            print(f"wrote synthetic {a.model} weights to {dst}")
            return 0
        from .ingest.keras_map import to_keras_variables
        from .ingest.savedmodel import write_savedmodel
        from .models import xception as X
        write_savedmodel(a.dst, to_keras_variables(X.init_params(seed=a.seed), residual_offset=a.residual_offset))
        print(f"wrote synthetic SavedModel to {a.dst}")
    elif a.cmd == "serve":
        from .serving.server import main as serve_main
        return serve_main(a.rest)
    return 0


if __name__ == "__main__":
    sys.exit(main())
