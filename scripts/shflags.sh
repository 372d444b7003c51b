#!/bin/bash
# gflags-style command-line flags for shell scripts -- this framework's
# equivalent of the vendored shflags the reference's launchers source
# (run.sh:3, run_lr2.sh:3).  Written from scratch; same calling
# convention so the reference's scripts port unchanged:
#
#   . ./scripts/shflags.sh
#   DEFINE_string  'job_name'   'ps'  'job name, ps or worker' 'j'
#   DEFINE_integer 'task_index' '0'   'task index'             'i'
#   DEFINE_float   'learning_rate' '0.001' 'learning rate'
#   DEFINE_boolean 'dry_run'    false 'print, do not run'
#   FLAGS "$@" || exit $?
#   eval set -- "${FLAGS_ARGV}"        # the non-flag arguments
#   echo "${FLAGS_job_name} ${FLAGS_task_index}"
#
# Accepted forms: --name=value, --name value, -s value, -svalue (short name),
# --bool / --nobool / --bool=true|false|1|0 for booleans, '--' ends the flags.
# Types are validated (integer, float, boolean).  --help / -h prints the flag
# table and makes FLAGS return 2 (FLAGS_HELP holds the text).  Multi-value
# flags (DEFINE_multi_*) accumulate every occurrence into a bash array
# FLAGS_<name>.  flags_reset forgets every definition.

__dtf_flag_names=()

_dtf_flags_define() {   # type name default help [short]
  local type=$1 name=$2 default=$3 help=$4 short=${5:-}
  if [ $# -lt 4 ]; then
    echo "flags: DEFINE_${type} needs: name default help [short]" >&2
    return 1
  fi
  case " ${__dtf_flag_names[*]} " in
    *" ${name} "*) echo "flags: flag '${name}' already defined" >&2; return 1 ;;
  esac
  if [[ ! ${name} =~ ^[A-Za-z_][A-Za-z0-9_]*$ ]]; then
    echo "flags: invalid flag name '${name}'" >&2
    return 1
  fi
  if [ "${type}" = boolean ]; then
    default=$(_dtf_flags_bool "${default}") || { echo "flags: bad boolean default for ${name}" >&2; return 1; }
  elif [[ ${type} != multi_* ]]; then
    _dtf_flags_check "${type}" "${default}" || { echo "flags: bad ${type} default for ${name}" >&2; return 1; }
  fi
  __dtf_flag_names+=("${name}")
  eval "__dtf_type_${name}=\"\${type}\""
  eval "__dtf_default_${name}=\"\${default}\""
  eval "__dtf_help_${name}=\"\${help}\""
  eval "__dtf_short_${name}=\"\${short}\""
  if [[ ${type} == multi_* ]]; then
    eval "FLAGS_${name}=()"
    [ -n "${default}" ] && eval "FLAGS_${name}=(\"\${default}\")"
  else
    eval "FLAGS_${name}=\"\${default}\""
  fi
  return 0
}

_dtf_flags_bool() {     # normalise a boolean spelling to true/false
  case "$1" in
    true|True|TRUE|t|1|yes|y) echo true ;;
    false|False|FALSE|f|0|no|n) echo false ;;
    *) return 1 ;;
  esac
}

_dtf_flags_check() {    # type value
  case "$1" in
    integer|multi_integer) [[ $2 =~ ^[-+]?[0-9]+$ ]] ;;
    float|multi_float) [[ $2 =~ ^[-+]?([0-9]+\.?[0-9]*|\.[0-9]+)([eE][-+]?[0-9]+)?$ ]] ;;
    *) return 0 ;;
  esac
}

_dtf_flags_by_short() { # short -> name
  local n s
  for n in "${__dtf_flag_names[@]}"; do
    eval "s=\${__dtf_short_${n}}"
    [ -n "${s}" ] && [ "${s}" = "$1" ] && { echo "${n}"; return 0; }
  done
  return 1
}

_dtf_flags_known() { case " ${__dtf_flag_names[*]} " in *" $1 "*) return 0 ;; esac; return 1; }

_dtf_flags_set() {      # name value
  local name=$1 value=$2 type
  eval "type=\${__dtf_type_${name}}"
  if [ "${type}" = boolean ]; then
    value=$(_dtf_flags_bool "${value}") || { echo "flags: --${name} expects a boolean, got '$2'" >&2; return 1; }
  fi
  if ! _dtf_flags_check "${type}" "${value}"; then
    echo "flags: --${name} expects ${type#multi_}, got '${value}'" >&2
    return 1
  fi
  if [[ ${type} == multi_* ]]; then
    eval "FLAGS_${name}+=(\"\${value}\")"
  else
    eval "FLAGS_${name}=\"\${value}\""
  fi
}

flags_help() {          # the flag table (what --help prints)
  local n t d h s
  echo "flags:"
  for n in "${__dtf_flag_names[@]}"; do
    eval "t=\${__dtf_type_${n}} d=\${__dtf_default_${n}} h=\${__dtf_help_${n}} s=\${__dtf_short_${n}}"
    if [ -n "${s}" ]; then
      printf '  -%s,--%s:  %s (default: %s, type: %s)\n' "${s}" "${n}" "${h}" "'${d}'" "${t}"
    else
      printf '  --%s:  %s (default: %s, type: %s)\n' "${n}" "${h}" "'${d}'" "${t}"
    fi
  done
}

FLAGS() {               # parse "$@"; sets FLAGS_<name> and FLAGS_ARGV; 2 after --help
  FLAGS_ARGV=''
  FLAGS_HELP=''
  local arg name value type rest=()
  local saw_multi=' '
  while [ $# -gt 0 ]; do
    arg=$1
    shift
    case "${arg}" in
      --) rest+=("$@"); break ;;
      -h|--help) FLAGS_HELP=$(flags_help); echo "${FLAGS_HELP}"; return 2 ;;
      --*=*) name=${arg%%=*}; name=${name#--}; value=${arg#*=} ;;
      --*)
        name=${arg#--}
        if _dtf_flags_known "${name}"; then
          eval "type=\${__dtf_type_${name}}"
          if [ "${type}" = boolean ]; then value=true
          elif [ $# -gt 0 ]; then value=$1; shift
          else echo "flags: --${name} needs a value" >&2; return 1
          fi
        elif [[ ${name} == no* ]] && _dtf_flags_known "${name#no}" &&
             eval "[ \"\${__dtf_type_${name#no}}\" = boolean ]"; then
          name=${name#no}; value=false
        else
          echo "flags: unknown flag --${name}" >&2; return 1
        fi ;;
      -?*)
        name=$(_dtf_flags_by_short "${arg:1:1}") || { echo "flags: unknown flag ${arg}" >&2; return 1; }
        eval "type=\${__dtf_type_${name}}"
        if [ ${#arg} -gt 2 ]; then value=${arg:2}
        elif [ "${type}" = boolean ]; then value=true
        elif [ $# -gt 0 ]; then value=$1; shift
        else echo "flags: ${arg} needs a value" >&2; return 1
        fi ;;
      *) rest+=("${arg}"); continue ;;
    esac
    _dtf_flags_known "${name}" || { echo "flags: unknown flag --${name}" >&2; return 1; }
    eval "type=\${__dtf_type_${name}}"
    if [[ ${type} == multi_* ]] && [[ ${saw_multi} != *" ${name} "* ]]; then
      eval "FLAGS_${name}=()"      # the first occurrence replaces the default
      saw_multi+="${name} "
    fi
    _dtf_flags_set "${name}" "${value}" || return 1
  done
  local a
  for a in "${rest[@]}"; do
    FLAGS_ARGV="${FLAGS_ARGV:+${FLAGS_ARGV} }'${a//\'/\'\\\'\'}'"
  done
  return 0
}

flags_reset() {         # forget every definition (tests, re-sourcing)
  local n
  for n in "${__dtf_flag_names[@]}"; do
    unset "FLAGS_${n}" "__dtf_type_${n}" "__dtf_default_${n}" "__dtf_help_${n}" "__dtf_short_${n}"
  done
  __dtf_flag_names=()
  FLAGS_ARGV=''
  FLAGS_HELP=''
}

DEFINE_string()  { _dtf_flags_define string "$@"; }
DEFINE_integer() { _dtf_flags_define integer "$@"; }
DEFINE_int()     { _dtf_flags_define integer "$@"; }
DEFINE_float()   { _dtf_flags_define float "$@"; }
DEFINE_boolean() { _dtf_flags_define boolean "$@"; }
DEFINE_bool()    { _dtf_flags_define boolean "$@"; }
DEFINE_multi_string()  { _dtf_flags_define multi_string "$@"; }
DEFINE_multi_integer() { _dtf_flags_define multi_integer "$@"; }
DEFINE_multi_float()   { _dtf_flags_define multi_float "$@"; }
