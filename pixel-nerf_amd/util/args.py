"""``util.args.parse_args`` (reference src/util/args.py:9-112): the callers' command line plus the
experiment config.

Same flags, defaults and post-processing as the reference:
  * ``-c/--conf -r/--resume --gpu_id -n/--name -F/--dataset_format -G/--exp_group_name --logs_path
    --checkpoints_path --visual_path --epochs --lr --gamma -D/--datadir -R/--ray_batch_size``,
    then the caller's ``callback(parser)`` extras (args.py:21-77);
  * ``-G`` nests the logs / checkpoints / visuals paths; the checkpoint and visual directories of
    ``--name`` are created (args.py:80-86);
  * ``expconf.conf`` maps ``config.<name>`` and ``datadir.<name>`` (args.py:87-101);
  * ``data.format`` of the conf fills ``--dataset_format`` (args.py:103-104);
  * ``--gpu_id "0 1"`` becomes ``[0, 1]`` (args.py:106).

Where expconf.conf is found: the reference reads it from its project root (two levels above
args.py).  Here the callers run from the reference checkout (their relative ``conf/...`` paths
resolve against the working directory), so it is looked up in ``$PNR_PROJECT_ROOT``, then the
working directory, then this repository's root; without one, ``default_conf`` and
``default_datadir`` apply, as the reference's ``get_string(..., default)`` does for a name it
does not list.  HOCON is read by pyhocon when it is importable, else by ``pnr.conf.parse_file``
(the subset the shipped conf/*.conf use); both give ``get_int/get_float/get_bool/get_string``
and ``conf["a.b"]`` access.
"""
import argparse
import os

from pnr.conf import Conf, parse_file as _parse_file


def _parse(path):
    try:
        from pyhocon import ConfigFactory   # the reference's parser, when present
    except ImportError:
        return _parse_file(path)
    return ConfigFactory.parse_file(path)


def _expconf_path():
    here = os.path.dirname(os.path.abspath(__file__))
    roots = [os.environ.get("PNR_PROJECT_ROOT"), os.getcwd(), os.path.dirname(os.path.dirname(here))]
    for root in roots:
        if root and os.path.isfile(os.path.join(root, "expconf.conf")):
            return os.path.join(root, "expconf.conf")
    return None


def parse_args(
    callback=None,
    training=False,
    default_conf="conf/default_mv.conf",
    default_expname="example",
    default_data_format="dvr",
    default_num_epochs=10000000,
    default_lr=1e-4,
    default_gamma=1.00,
    default_datadir="data",
    default_ray_batch_size=50000,
    argv=None,
):
    """Returns ``(args, conf)`` as the reference does.  ``argv`` (not in the reference) parses an
    explicit list instead of ``sys.argv[1:]``."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--conf", "-c", type=str, default=None)
    ap.add_argument("--resume", "-r", action="store_true", help="continue training")
    ap.add_argument("--gpu_id", type=str, default="0", help="GPU(s) to use, space delimited")
    ap.add_argument("--name", "-n", type=str, default=default_expname, help="experiment name")
    ap.add_argument("--dataset_format", "-F", type=str, default=None,
                    help="Dataset format, multi_obj | dvr | dvr_gen | dvr_dtu | srn")
    ap.add_argument("--exp_group_name", "-G", type=str, default=None,
                    help="if we want to group some experiments together")
    ap.add_argument("--logs_path", type=str, default="logs", help="logs output directory")
    ap.add_argument("--checkpoints_path", type=str, default="checkpoints", help="checkpoints output directory")
    ap.add_argument("--visual_path", type=str, default="visuals", help="visualization output directory")
    ap.add_argument("--epochs", type=int, default=default_num_epochs, help="number of epochs to train for")
    ap.add_argument("--lr", type=float, default=default_lr, help="learning rate")
    ap.add_argument("--gamma", type=float, default=default_gamma, help="learning rate decay factor")
    ap.add_argument("--datadir", "-D", type=str, default=None, help="Dataset directory")
    ap.add_argument("--ray_batch_size", "-R", type=int, default=default_ray_batch_size, help="Ray batch size")
    if callback is not None:
        ap = callback(ap)
    args = ap.parse_args(argv)

    if args.exp_group_name is not None:
        args.logs_path = os.path.join(args.logs_path, args.exp_group_name)
        args.checkpoints_path = os.path.join(args.checkpoints_path, args.exp_group_name)
        args.visual_path = os.path.join(args.visual_path, args.exp_group_name)
    os.makedirs(os.path.join(args.checkpoints_path, args.name), exist_ok=True)
    os.makedirs(os.path.join(args.visual_path, args.name), exist_ok=True)

    exp_path = _expconf_path()
    expconf = _parse(exp_path) if exp_path else Conf({})
    if args.conf is None:
        args.conf = expconf.get_string("config." + args.name, default_conf)
    if args.datadir is None:
        args.datadir = expconf.get_string("datadir." + args.name, default_datadir)
    conf = _parse(args.conf)
    if args.dataset_format is None:
        args.dataset_format = conf.get_string("data.format", default_data_format)
    args.gpu_id = list(map(int, args.gpu_id.split()))

    print("EXPERIMENT NAME:", args.name)
    if training:
        print("CONTINUE?", "yes" if args.resume else "no")
    print("* Config file:", args.conf)
    print("* Dataset format:", args.dataset_format)
    print("* Dataset location:", args.datadir)
    return args, conf
