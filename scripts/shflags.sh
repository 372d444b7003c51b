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
# Types are validated (integer, float, boolean).  Multi-value flags
# (DEFINE_multi_*) accumulate every occurrence into a bash array FLAGS_<name>.
# flags_reset forgets every definition.
#
# Help surface (reference shflags:1842-2097): --help / -h (usage, description,
# flag table), --helpshort (usage + flag names only), --helpxml (XML flag
# dump), --helpman (roff man page on stdout), --version (HELP_VERSION).  Each
# makes FLAGS print and return 2 (FLAGS_HELP holds the text).  Optional
# HELP_COMMAND / HELP_VERSION / HELP_DESCRIPTION / HELP_CONTACT /
# HELP_COPYRIGHT variables fill the texts.  Flags defined with a trailing
# 'required' category (DEFINE_string name default help short required) must be
# given on the command line.
#
# Parsing is pure bash, so long flags work whatever getopt(1) the system has;
# flags_getoptIsEnh / flags_getoptIsStd / flags_getoptInfo still report the
# system getopt flavour (enhanced = util-linux `getopt -T` exits 4) for scripts
# that branch on it.

[ -n "${FLAGS_VERSION:-}" ] && [ -n "${__dtf_flags_loaded:-}" ] && return 0
__dtf_flags_loaded=1
FLAGS_VERSION='1.0.5'       # API level of the shflags surface reproduced here
FLAGS_TRUE=0
FLAGS_FALSE=1
FLAGS_ERROR=2
__dtf_flag_names=()

_dtf_flags_define() {   # type name default help [short] [required]
  local type=$1 name=$2 default=$3 help=$4 short=${5:-} cat=${6:-}
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
  eval "__dtf_required_${name}=$([ "${cat}" = required ] && echo 1 || echo 0)"
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

_dtf_flags_command() { echo "${HELP_COMMAND:-${FLAGS_PARENT:-${0##*/}}}"; }

flags_usage() {         # synopsis: required flags bare, optional ones in brackets
  local n s u line
  line="USAGE: $(_dtf_flags_command)"
  for n in "${__dtf_flag_names[@]}"; do
    eval "s=\${__dtf_short_${n}} u=\${__dtf_required_${n}}"
    local f="--${n}"
    [ -n "${s}" ] && f="-${s}|--${n}"
    if [ "${u}" = 1 ]; then line+=" ${f}"; else line+=" [${f}]"; fi
  done
  echo "${line} [args]"
}

flags_helpshort() {     # usage + flag names and types, no descriptions
  local n t s
  flags_usage
  echo "flags:"
  for n in "${__dtf_flag_names[@]}"; do
    eval "t=\${__dtf_type_${n}} s=\${__dtf_short_${n}}"
    if [ -n "${s}" ]; then printf '  -%s,--%s (%s)\n' "${s}" "${n}" "${t}"
    else printf '  --%s (%s)\n' "${n}" "${t}"
    fi
  done
}

flags_help() {          # usage, description and the flag table (what --help prints)
  local n t d h s u
  flags_usage
  [ -n "${HELP_DESCRIPTION:-}" ] && printf '%s\n' "${HELP_DESCRIPTION}"
  echo "flags:"
  for n in "${__dtf_flag_names[@]}"; do
    eval "t=\${__dtf_type_${n}} d=\${__dtf_default_${n}} h=\${__dtf_help_${n}} s=\${__dtf_short_${n}}"
    eval "u=\${__dtf_required_${n}}"
    [ "${u}" = 1 ] && h="${h} [required]"
    if [ -n "${s}" ]; then
      printf '  -%s,--%s:  %s (default: %s, type: %s)\n' "${s}" "${n}" "${h}" "'${d}'" "${t}"
    else
      printf '  --%s:  %s (default: %s, type: %s)\n' "${n}" "${h}" "'${d}'" "${t}"
    fi
  done
}

_dtf_xml() {            # XML-escape $1
  local v=${1//&/&amp;}
  v=${v//</&lt;}; v=${v//>/&gt;}; v=${v//\"/&quot;}
  printf '%s' "${v}"
}

flags_helpxml() {       # machine-readable flag dump
  local n t d h s u
  echo '<?xml version="1.0"?>'
  echo '<AllFlags>'
  echo "  <name>$(_dtf_xml "$(_dtf_flags_command)")</name>"
  echo "  <version>$(_dtf_xml "${HELP_VERSION:-unknown}")</version>"
  echo "  <description>$(_dtf_xml "${HELP_DESCRIPTION:-}")</description>"
  for n in "${__dtf_flag_names[@]}"; do
    eval "t=\${__dtf_type_${n}} d=\${__dtf_default_${n}} h=\${__dtf_help_${n}} s=\${__dtf_short_${n}}"
    eval "u=\${__dtf_required_${n}}"
    echo '  <flag>'
    echo "    <category>$([ "${u}" = 1 ] && echo required || echo optional)</category>"
    echo "    <name>$(_dtf_xml "${n}")</name>"
    echo "    <short_name>$(_dtf_xml "${s}")</short_name>"
    echo "    <meaning>$(_dtf_xml "${h}")</meaning>"
    echo "    <default>$(_dtf_xml "${d}")</default>"
    echo "    <current>$(_dtf_xml "$(eval "echo \"\${FLAGS_${n}[*]}\"")")</current>"
    echo "    <type>${t}</type>"
    echo '  </flag>'
  done
  echo '</AllFlags>'
}

flags_helpman() {       # man(7) page on stdout (pipe to `man -l -`)
  local n t d h s cmd
  cmd=$(_dtf_flags_command)
  echo ".TH \"$(echo "${cmd}" | tr '[:lower:]' '[:upper:]')\" 1 \"\" \"${HELP_VERSION:-}\""
  echo '.SH NAME'
  echo "${cmd}"
  echo '.SH SYNOPSIS'
  flags_usage | sed 's/^USAGE: //'
  if [ -n "${HELP_DESCRIPTION:-}" ]; then echo '.SH DESCRIPTION'; printf '%s\n' "${HELP_DESCRIPTION}"; fi
  echo '.SH OPTIONS'
  for n in "${__dtf_flag_names[@]}"; do
    eval "t=\${__dtf_type_${n}} d=\${__dtf_default_${n}} h=\${__dtf_help_${n}} s=\${__dtf_short_${n}}"
    echo '.TP'
    if [ -n "${s}" ]; then echo "\\fB\\-${s}\\fR, \\fB\\-\\-${n}\\fR"; else echo "\\fB\\-\\-${n}\\fR"; fi
    echo "${h} (default: ${d}; type: ${t})"
  done
  [ -n "${HELP_CONTACT:-}" ] && { echo '.SH CONTACT'; printf '%s\n' "${HELP_CONTACT}"; }
  [ -n "${HELP_COPYRIGHT:-}" ] && { echo '.SH COPYRIGHT'; printf '%s\n' "${HELP_COPYRIGHT}"; }
  return 0
}

flags_version() { echo "$(_dtf_flags_command) ${HELP_VERSION:-unknown}"; }

# system getopt flavour: util-linux (enhanced, long options) returns 4 for -T
__dtf_getopt_enh() { ${FLAGS_GETOPT_CMD:-getopt} -T >/dev/null 2>&1; [ $? -eq 4 ]; }
flags_getoptIsEnh() { __dtf_getopt_enh; }
flags_getoptIsStd() { ! __dtf_getopt_enh; }
flags_getoptInfo() {
  echo "flags:DEBUG shell: bash ${BASH_VERSION}" >&2
  echo "flags:DEBUG getopt: $(${FLAGS_GETOPT_CMD:-getopt} --version 2>&1 | head -1)" >&2
  echo "flags:DEBUG getopt flavour: $(__dtf_getopt_enh && echo enhanced || echo standard)" >&2
  echo "flags:DEBUG parser: built-in (long flags on any getopt)" >&2
}

FLAGS() {               # parse "$@"; sets FLAGS_<name> and FLAGS_ARGV; 2 after --help
  FLAGS_ARGV=''
  FLAGS_HELP=''
  local arg name value type rest=()
  local saw_multi=' ' given=' '
  while [ $# -gt 0 ]; do
    arg=$1
    shift
    case "${arg}" in
      --) rest+=("$@"); break ;;
      -h|--help) FLAGS_HELP=$(flags_help); echo "${FLAGS_HELP}"; return 2 ;;
      --helpshort) FLAGS_HELP=$(flags_helpshort); echo "${FLAGS_HELP}"; return 2 ;;
      --helpxml) FLAGS_HELP=$(flags_helpxml); echo "${FLAGS_HELP}"; return 2 ;;
      --helpman) FLAGS_HELP=$(flags_helpman); echo "${FLAGS_HELP}"; return 2 ;;
      --version) FLAGS_HELP=$(flags_version); echo "${FLAGS_HELP}"; return 2 ;;
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
    given+="${name} "
  done
  local a
  for a in "${rest[@]}"; do
    FLAGS_ARGV="${FLAGS_ARGV:+${FLAGS_ARGV} }'${a//\'/\'\\\'\'}'"
  done
  local u missing=''
  for name in "${__dtf_flag_names[@]}"; do
    eval "u=\${__dtf_required_${name}}"
    [ "${u}" = 1 ] && [[ ${given} != *" ${name} "* ]] && missing+=" --${name}"
  done
  if [ -n "${missing}" ]; then
    echo "flags: missing required flag(s):${missing}" >&2
    return 1
  fi
  return 0
}

flags_reset() {         # forget every definition (tests, re-sourcing)
  local n
  for n in "${__dtf_flag_names[@]}"; do
    unset "FLAGS_${n}" "__dtf_type_${n}" "__dtf_default_${n}" "__dtf_help_${n}" "__dtf_short_${n}" \
      "__dtf_required_${n}"
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
