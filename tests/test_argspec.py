"""The operands' argparse-free command line (cli/argspec.py) and lazy logging
(utils/logs.py): the fast parser's result equals argparse's on every command
the operator renders, and on the forms it hands back to argparse."""

import os
import subprocess
import sys

import pytest

from amdgpu_operator.cli.argspec import Spec
from amdgpu_operator.cli.operands import _split_passthrough, build_parser, operand_spec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _both(argv):
    spec = operand_spec()
    fast = spec._fast(list(argv))
    ref = build_parser().parse_args(argv)
    return fast, ref


def _rendered_commands(flags):
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags, spec_from_values
    from amdgpu_operator.controller import manifests as MF

    spec = spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + flags))
    for builder in MF.STATE_BUILDERS.values():
        for o in builder(spec, "ns", None):
            if o.get("kind") not in ("DaemonSet", "Deployment", "Job"):
                continue
            tmpl = o["spec"]["template"]["spec"]
            for c in tmpl.get("initContainers", []) + tmpl["containers"]:
                if c.get("command") == ["amdgpu-operator"]:
                    yield list(c["args"])


@pytest.mark.parametrize("flags", [[], ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true",
                                        "sandboxWorkloads.enabled=true", "migManager.enabled=true"],
                                   ["devicePlugin.partitionStrategy=mixed", "validator.pluginPods=perDevice",
                                    "validator.pluginPodCheck=hip"]])
def test_fast_parse_equals_argparse_on_rendered_commands(flags):
    n = 0
    for args in _rendered_commands(flags):
        if args[0] == "validate":
            known, _ = _split_passthrough(args[1:])
            args = ["validate", *known]
        if args[0] not in operand_spec().commands:
            continue  # the operator's own sub-commands (cli/main.py)
        fast, ref = _both(args)
        assert fast is not None, args  # the rendered forms never need argparse
        assert vars(fast) == vars(ref), args
        n += 1
    assert n >= 5


@pytest.mark.parametrize("argv", [
    ["driver", "install"],
    ["driver", "monitor", "--interval", "2.5"],
    ["driver", "monitor", "--interval=3"],
    ["toolkit", "install", "--runtime-class", "amd", "--no-cdi"],
    ["validate", "gpu", "--with-driver", "--complete", "--timeout", "30", "--pod-check", "hip"],
    ["device-plugin", "--device-list-strategy", "envvar,cdi-cri", "--health-poll-ms", "250", "--cdi"],
    ["metrics-exporter", "--port", "9500", "--pod-attribution"],
    ["nfd", "--oneshot"],
    ["partition-manager", "--default-compute", "CPX"],
    ["vfio-manager", "bind", "--kfd-idle-timeout", "5"],
    ["dra-driver"],
    ["sandbox-device-plugin", "--resource-prefix", "example.com"],
    ["gfd", "--interval", "7", "--label-prefix", "x.io"],
])
def test_fast_parse_equals_argparse(argv):
    fast, ref = _both(argv)
    assert fast is not None and vars(fast) == vars(ref)


@pytest.mark.parametrize("argv", [
    ["driver", "monitor", "--interv", "2"],        # an abbreviation: argparse's
    ["driver", "monitor", "--interval", "-1"],     # a negative number: argparse's
    ["nfd", "--interval", "1e1"],                  # float() takes it; same either way
])
def test_forms_handed_to_argparse_parse_the_same(argv):
    ref = build_parser().parse_args(argv)
    assert vars(operand_spec().parse(argv)) == vars(ref)


@pytest.mark.parametrize("argv", [
    ["driver", "bogus"],                       # not a choice
    ["driver", "install", "--no-such-flag"],
    ["validate", "gpu", "--timeout", "soon"],  # not a float
    ["toolkit"],                               # positional missing
    ["nope"],
])
def test_bad_command_lines_fail_like_argparse(argv, capsys):
    with pytest.raises(SystemExit) as e:
        operand_spec().parse(argv)
    assert e.value.code == 2
    assert "error" in capsys.readouterr().err


def test_help_is_argparse_help(capsys):
    with pytest.raises(SystemExit) as e:
        operand_spec().parse(["driver", "--help"])
    assert e.value.code == 0 and "prepare-upgrade" in capsys.readouterr().out


def test_string_defaults_are_converted_like_argparse():
    s = Spec(prog="x")
    c = s.add_subparsers(dest="cmd", required=True).add_parser("run")
    c.add_argument("--n", type=int, default="7")
    c.add_argument("--flag", action="store_true")
    fast = s._fast(["run"])
    assert vars(fast) == vars(s.argparse().parse_args(["run"])) == {"cmd": "run", "n": 7, "flag": False}


def test_operand_start_path_imports_neither_argparse_nor_logging():
    """What `python3 -S -m amdgpu_operator <operand>` loads before the
    operand runs: the entry point, the client, the node environment, and
    the driver / toolkit / validator modules."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import amdgpu_operator.cli.main, amdgpu_operator.cli.operands, amdgpu_operator.kube.client\n"
            "import amdgpu_operator.nodeenv, amdgpu_operator.validator.validate, amdgpu_operator.driver.manager\n"
            "import amdgpu_operator.toolkit.install\n"
            "from amdgpu_operator.cli.operands import operand_spec\n"
            "operand_spec().parse(['validate', 'gpu', '--with-driver', '--complete'])\n"
            "print(sorted(m for m in ('argparse', 'logging', 'dataclasses', 'inspect') if m in sys.modules))\n" % ROOT)
    out = subprocess.run([sys.executable, "-S", "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "[]"


def test_lazy_logging_applies_setup_at_first_use():
    """setup() before logging is loaded takes effect at the first log call:
    one JSON record on stderr, at the configured level."""
    code = ("import sys, json; sys.path.insert(0, %r)\n"
            "from amdgpu_operator.utils import logs\n"
            "log = logs.get_logger('amdgpu.test')\n"
            "logs.setup('warning')\n"
            "assert 'logging' not in sys.modules\n"
            "log.info('hidden')\n"
            "log.warning('shown %%d', 3, extra={'node': 'n1'})\n" % ROOT)
    out = subprocess.run([sys.executable, "-S", "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stderr.splitlines() if ln.strip()]
    assert len(lines) == 1
    import json

    rec = json.loads(lines[0])
    assert rec["msg"] == "shown 3" and rec["level"] == "warning" and rec["node"] == "n1" and rec["logger"] == "amdgpu.test"
