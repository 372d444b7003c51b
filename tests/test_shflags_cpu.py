"""scripts/shflags.sh (the shell flag library) and the shell entry
points built on it (scripts/run.sh, scripts/run_lr2.sh)."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "scripts", "shflags.sh")


def _bash(body, *args):
    script = f". {LIB}\n{body}"
    return subprocess.run(["bash", "-c", script, "test"] + list(args), capture_output=True, text=True, timeout=30)


DEFS = """
DEFINE_string 'job_name' 'ps' 'job name' 'j'
DEFINE_integer 'task_index' '0' 'task index' 'i'
DEFINE_float 'learning_rate' '0.001' 'lr'
DEFINE_boolean 'verbose' false 'chatty' 'v'
DEFINE_multi_string 'tag' '' 'tags'
"""


def test_defaults_and_long_short_forms():
    r = _bash(DEFS + 'FLAGS "$@" || exit $?\neval set -- "${FLAGS_ARGV}"\n'
              'echo "$FLAGS_job_name|$FLAGS_task_index|$FLAGS_learning_rate|$FLAGS_verbose|$#|$1|$2"',
              "--job_name=worker", "-i", "3", "--learning_rate", "0.5", "-v", "pos 1", "--", "--not-a-flag")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "worker|3|0.5|true|2|pos 1|--not-a-flag"
    r = _bash(DEFS + 'FLAGS "$@" || exit $?\necho "$FLAGS_job_name|$FLAGS_task_index|$FLAGS_verbose"')
    assert r.stdout.strip() == "ps|0|false"


def test_boolean_negation_and_multi():
    r = _bash(DEFS + 'FLAGS "$@" || exit $?\necho "$FLAGS_verbose ${#FLAGS_tag[@]} ${FLAGS_tag[*]}"',
              "--verbose", "--noverbose", "--tag=a", "--tag", "b c")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "false 2 a b c"


def test_type_validation_and_unknown_flags():
    r = _bash(DEFS + 'FLAGS "$@"', "--task_index=abc")
    assert r.returncode == 1 and "expects integer" in r.stderr
    r = _bash(DEFS + 'FLAGS "$@"', "--learning_rate=1e-3")
    assert r.returncode == 0, r.stderr
    r = _bash(DEFS + 'FLAGS "$@"', "--bogus=1")
    assert r.returncode == 1 and "unknown flag" in r.stderr
    r = _bash("DEFINE_integer 'n' 'x' 'bad default'")
    assert r.returncode == 1


def test_help_and_reset():
    r = _bash(DEFS + 'FLAGS "$@"; echo "rc=$?"', "--help")
    assert "-j,--job_name:  job name (default: 'ps', type: string)" in r.stdout
    assert "rc=2" in r.stdout
    r = _bash(DEFS + "flags_reset\nDEFINE_string 'job_name' 'x' 'again'\nFLAGS\necho $FLAGS_job_name")
    assert r.returncode == 0 and r.stdout.strip() == "x"


def test_run_lr2_dry_run():
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "run_lr2.sh"), "--train=/tmp/a", "-T", "/tmp/b",
                        "--run_mode=test", "--job_name=worker", "-i", "1", "--dry_run"],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "distributed_tensorflow_example_amd.launch lr2" in out
    assert "--job_name=worker" in out and "--task_index=1" in out and "--run_mode=test" in out


def test_run_sh_writes_file_lists(tmp_path):
    for kind in ("train", "test"):
        d = tmp_path / kind
        d.mkdir()
        for i in range(3):
            (d / f"part-{i:05d}").write_text("1 3:1.0\n" * 10)
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "run.sh"), f"--train={tmp_path / 'train'}",
                        f"--test={tmp_path / 'test'}", f"--train_file_list={tmp_path / 'tl'}",
                        f"--test_file_list={tmp_path / 'sl'}"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = (tmp_path / "tl").read_text().split()
    assert len(lines) == 3 and all("part-" in l for l in lines)


def test_help_variants_version_and_required():
    defs = DEFS + "DEFINE_string 'train' '' 'training files' 't' required\n"
    env_txt = "HELP_VERSION=2.1\nHELP_DESCRIPTION='Sparse LR launcher'\nHELP_COMMAND=run_lr2\n"
    r = _bash(env_txt + defs + 'FLAGS "$@"; echo "rc=$?"', "--helpshort")
    assert "USAGE: run_lr2 [-j|--job_name]" in r.stdout and "-t|--train" in r.stdout
    assert "  -j,--job_name (string)" in r.stdout and "job name" not in r.stdout and "rc=2" in r.stdout
    r = _bash(env_txt + defs + 'FLAGS "$@"; echo "rc=$?"', "--version")
    assert r.stdout.splitlines()[0] == "run_lr2 2.1" and "rc=2" in r.stdout
    r = _bash(env_txt + defs + 'FLAGS "$@"', "--helpxml")
    import xml.etree.ElementTree as ET
    root = ET.fromstring(r.stdout)
    assert root.find("name").text == "run_lr2" and root.find("version").text == "2.1"
    flags = {f.find("name").text: f for f in root.findall("flag")}
    assert flags["train"].find("category").text == "required"
    assert flags["task_index"].find("default").text == "0" and flags["task_index"].find("type").text == "integer"
    r = _bash(env_txt + defs + 'FLAGS "$@"', "--helpman")
    assert r.stdout.startswith('.TH "RUN_LR2" 1') and ".SH OPTIONS" in r.stdout and "Sparse LR launcher" in r.stdout
    r = _bash(env_txt + defs + 'FLAGS "$@"; echo "rc=$?"', "--job_name=worker")
    assert "rc=1" in r.stdout and "missing required flag(s): --train" in r.stderr
    r = _bash(env_txt + defs + 'FLAGS "$@" && echo "ok $FLAGS_train"', "-t", "/data/a")
    assert r.stdout.strip() == "ok /data/a", r.stderr
    r = _bash(env_txt + defs + 'FLAGS "$@"; echo "rc=$?"', "--help")
    assert "Sparse LR launcher" in r.stdout and "training files [required]" in r.stdout


def test_getopt_introspection():
    r = _bash('if flags_getoptIsEnh; then echo enh; fi; if flags_getoptIsStd; then echo std; fi; '
              'flags_getoptInfo; echo "v=$FLAGS_VERSION"')
    out = r.stdout.split()
    assert (("enh" in out) != ("std" in out)) and "v=1.0.5" in out
    assert "flags:DEBUG parser: built-in" in r.stderr
