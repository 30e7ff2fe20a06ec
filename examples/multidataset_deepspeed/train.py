"""Multi-dataset GFM training with the DeepSpeed engine's features (reference
``examples/multidataset_deepspeed/{train.py, base.json}``: ``deepspeed.initialize`` with
``--zero_opt`` -> ZeRO stage 1, optional bf16, otherwise the multidataset driver).

DeepSpeed is not part of this framework: its two features the reference
example uses map onto native pieces —
  ``--zero_opt``  -> ``Optimizer.use_zero_redundancy`` (flat element-sharded ZeRO-1:
                    reduce-scatter of gradients, sharded AdamW state, all-gather of
                    parameters; ``hydragnn_amd/parallel/zero.py``);
  ``--bf16``      -> ``Training.precision = "bf16"`` (bf16 MFMA GEMMs, fp32 master
                    weights / accumulation).
Everything else (stores, --multi / --ddstore / --shmem, rank assignment) is the
``examples/multidataset/train.py`` driver, run with the derived config.

Usage: torchrun --nproc-per-node 4 examples/multidataset_deepspeed/train.py --zero_opt [--bf16] [multidataset flags]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "multidataset"))
sys.path.insert(0, os.path.dirname(HERE))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    zero = "--zero_opt" in argv
    bf16 = "--bf16" in argv
    argv = [a for a in argv if a not in ("--zero_opt", "--bf16")]
    src = "base.json"
    if "--inputfile" in argv:
        i = argv.index("--inputfile")
        src = argv[i + 1]
        del argv[i:i + 2]
    path = src if os.path.isabs(src) else os.path.join(HERE, src)
    with open(path) as f:
        config = json.load(f)
    tr = config["NeuralNetwork"]["Training"]
    tr["Optimizer"]["use_zero_redundancy"] = zero
    if bf16:
        tr["precision"] = "bf16"
    workdir = os.path.abspath(argv[argv.index("--workdir") + 1]) if "--workdir" in argv else os.getcwd()
    os.makedirs(workdir, exist_ok=True)
    rank = os.environ.get("RANK", "0")
    derived = os.path.join(workdir, f"deepspeed_derived_config_rank{rank}.json")
    with open(derived, "w") as f:
        json.dump(config, f, indent=1)
    import train as gfm  # examples/multidataset/train.py

    return gfm.main(argv + ["--inputfile", derived])


if __name__ == "__main__":
    main()
