"""Pack a saved inference model into one "merged model" buffer for the C-API's
``paddle_gradient_machine_create_for_inference_with_parameters`` (reference
python/paddle/utils/merge_model.py, which packs a ModelConfig and its parameters):

    "PAMERGE1" | uint64 len | ProgramDesc bytes | uint64 len | combined parameter stream

``python -m paddle_amd.utils.merge_model MODEL_DIR OUT [PARAMS_FILENAME]``."""
import os
import struct
import sys
import tempfile


def merge_model(model_dir, output_file, params_filename=None, model_filename=None):
    prog_path = os.path.join(model_dir, model_filename or "__model__")
    with open(prog_path, "rb") as f:
        prog = f.read()
    if params_filename:
        with open(os.path.join(model_dir, params_filename), "rb") as f:
            params = f.read()
    else:
        # per-variable files: re-save the same program with one combined stream
        from .. import fluid

        exe = fluid.Executor(fluid.CPUPlace())
        with fluid.executor.scope_guard(fluid.core.Scope()):
            p, feeds, fetches = fluid.io.load_inference_model(model_dir, exe, model_filename=model_filename)
            with tempfile.TemporaryDirectory() as d:
                fluid.io.save_inference_model(d, feeds, fetches, exe, main_program=p, params_filename="params")
                with open(os.path.join(d, "__model__"), "rb") as f:
                    prog = f.read()
                with open(os.path.join(d, "params"), "rb") as f:
                    params = f.read()
    with open(output_file, "wb") as f:
        f.write(b"PAMERGE1" + struct.pack("<Q", len(prog)) + prog + struct.pack("<Q", len(params)) + params)
    return output_file


if __name__ == "__main__":
    if len(sys.argv) not in (3, 4):
        print(__doc__, file=sys.stderr)
        sys.exit(2)
    merge_model(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) == 4 else None)
