#!/bin/bash
# Shell entry point that writes the train/test file lists (the reference's
# run.sh): lists every file under --train / --test (local or
# hdfs:// via the gfile registry) and writes them, one per line, to
# --train_file_list / --test_file_list (any gfile path).
HERE=$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)
. "${HERE}/shflags.sh"

DEFINE_string 'train' '' 'train data path' 't'
DEFINE_string 'test' '' 'test data path' 'T'
DEFINE_string 'train_file_list' '' 'where to write the train file list'
DEFINE_string 'test_file_list' '' 'where to write the test file list'

FLAGS "$@" || exit $?
eval set -- "${FLAGS_ARGV}"
for kind in train test; do
  src_var="FLAGS_${kind}"; out_var="FLAGS_${kind}_file_list"
  if [ -z "${!src_var}" ] || [ -z "${!out_var}" ]; then
    echo "run.sh: --${kind} and --${kind}_file_list are required" >&2
    flags_help >&2
    exit 1
  fi
done
cd "${HERE}/.." || exit 1
export PYTHONPATH="${PWD}${PYTHONPATH:+:${PYTHONPATH}}"
python -m distributed_tensorflow_example_amd.launch filelist "${FLAGS_train}" --sep newline --out "${FLAGS_train_file_list}" &&
python -m distributed_tensorflow_example_amd.launch filelist "${FLAGS_test}" --sep newline --out "${FLAGS_test_file_list}"
