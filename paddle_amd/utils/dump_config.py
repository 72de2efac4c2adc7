"""Print a v1 config's ModelConfig (reference python/paddle/utils/dump_config.py):

    python -m paddle_amd.utils.dump_config CONFIG.py [CONFIG_ARG_STR] [--whole | --binary]

text format of the ModelConfig (default), of the whole TrainerConfig (``--whole``),
or the serialised ModelConfig bytes (``--binary``), from the DSL's parse_config
(trainer_config_helpers/config_proto.py)."""
import sys


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not 1 <= len(argv) <= 3:
        print(__doc__, file=sys.stderr)
        return 2
    from ..trainer_config_helpers import config_proto as cp
    from ..trainer_config_helpers import parse_config

    conf = parse_config(argv[0], argv[1] if len(argv) > 1 else "")
    mode = argv[2] if len(argv) > 2 else ""
    if mode == "--whole":
        sys.stdout.write(conf.to_text(whole=True))
    elif mode == "--binary":
        sys.stdout.buffer.write(cp.encode("ModelConfig", conf.model_config()))
    else:
        sys.stdout.write(conf.to_text())
    return 0


if __name__ == "__main__":
    sys.exit(main())
