#!/bin/bash
# Shell entry point of the sparse-LR job (the reference's run_lr2.sh):
# gflags-style flags (scripts/shflags.sh), input file lists from any gfile
# path (local, hdfs://), then either a whole local ps/worker cluster on this
# node's GPUs (run_mode=product; the reference submitted to an external
# tf_tool cluster) or one task (run_mode=test).
HERE=$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)
. "${HERE}/shflags.sh"

DEFINE_string 'job_name' 'ps' 'job name, ps or worker' 'j'
DEFINE_integer 'task_index' '0' 'task index' 'i'
DEFINE_string 'train' '' 'train data path (dir, glob or file; hdfs:// supported)' 't'
DEFINE_string 'test' '' 'test data path' 'T'
DEFINE_string 'run_mode' 'product' 'run mode, product or test'
DEFINE_string 'output' '' 'output root path (checkpoints)'
DEFINE_string 'load_mode' 'queue' 'load mode, all or queue'
DEFINE_float 'learning_rate' '0.001' 'learning rate'
DEFINE_integer 'num_epochs' 120 'number of epochs'
DEFINE_integer 'batch_size' 500 'batch size'
DEFINE_integer 'features' 4762348 'feature count'
DEFINE_integer 'num_workers' 1 'product mode: worker processes (one GPU each)'
DEFINE_string 'gpus' '' 'product mode: comma list of GPU ids for the workers'
DEFINE_boolean 'dry_run' false 'print the launcher command, do not run it'

FLAGS "$@" || exit $?
eval set -- "${FLAGS_ARGV}"
if [ -z "${FLAGS_train}" ] || [ -z "${FLAGS_test}" ]; then
  echo "run_lr2.sh: --train and --test are required" >&2
  flags_help >&2
  exit 1
fi

cmd=(python -m distributed_tensorflow_example_amd.launch lr2
     --job_name="${FLAGS_job_name}" --task_index="${FLAGS_task_index}"
     --train="${FLAGS_train}" --test="${FLAGS_test}" --run_mode="${FLAGS_run_mode}"
     --load_mode="${FLAGS_load_mode}" --learning_rate="${FLAGS_learning_rate}"
     --num_epochs="${FLAGS_num_epochs}" --batch_size="${FLAGS_batch_size}" --features="${FLAGS_features}"
     --num_workers="${FLAGS_num_workers}")
[ -n "${FLAGS_output}" ] && cmd+=(--output="${FLAGS_output}")
[ -n "${FLAGS_gpus}" ] && cmd+=(--gpus="${FLAGS_gpus}")
[ $# -gt 0 ] && cmd+=(-- "$@")

if [ "${FLAGS_dry_run}" = true ]; then
  printf '%q ' "${cmd[@]}"; echo
  exit 0
fi
cd "${HERE}/.." && PYTHONPATH="${PWD}${PYTHONPATH:+:${PYTHONPATH}}" exec "${cmd[@]}"
