(* OCaml ctypes bindings of libcpr_hip (include/cpr_hip.h, CPR_ABI_VERSION 11).

   For a host that has OCaml: dropped next to the reference's gym engine
   (simulator/gym/), it lets Hip_engine.of_module (hip_engine.ml) stand in for
   Engine.of_module (simulator/gym/engine.ml:97-273). Field order and C types follow
   include/cpr_hip.h exactly; Ctypes computes the C layout (padding included).

   Not compiled in this repository: its build image has no OCaml toolchain (SURVEY.md
   8c). tests/test_host.py checks that every field and function named here exists in the
   header with the same order. *)

open Ctypes
open Foreign

let abi_version = 11

(* ---- status codes and enums (cpr_status, cpr_protocol, cpr_network, cpr_mode) *)
let ok = 0
let e_invalid_arg = -1
let e_unsupported = -2
let e_hip = -3
let e_capacity = -4
let e_state = -5
let proto_nakamoto = 0l
let proto_ethereum = 1l
let proto_bk = 2l
let proto_tailstorm = 3l
let proto_fc16 = 4l
let net_selfish_mining = 0l
let net_two_agents = 1l
let net_honest_clique = 2l
let net_exp_clique = 3l
let net_abstract_gamma = 4l (* flagged abstract-gamma mode, not a reference network *)
let mode_gym = 0l
let mode_loop = 1l

(* cpr_episode_status bits *)
let st_tie = 1l
let st_overlap = 2l
let st_deep_fork = 4l
let st_tie_unresolved = 8l
let st_stale_time = 16l
let st_capacity = 32l
let st_reference_raises = 64l
let st_trace_miss = 128l
let st_exact_rerun = 256l
let st_invalid = Int32.(logor st_capacity (logor st_reference_raises st_trace_miss))

let st_lockstep_inexact =
  Int32.(logor st_overlap (logor st_deep_fork (logor st_tie_unresolved st_stale_time)))
;;

(* ---- opaque handles *)
type ctx
type batch

let ctx : ctx structure typ = structure "cpr_ctx"
let batch : batch structure typ = structure "cpr_batch"

(* ---- cpr_config *)
type config

let config : config structure typ = structure "cpr_config"
let c_protocol = field config "protocol" int32_t
let c_network = field config "network" int32_t
let c_mode = field config "mode" int32_t
let c_policy = field config "policy" int32_t
let c_policy_table = field config "policy_table" (ptr uint8_t)
let c_policy_table_dim = field config "policy_table_dim" int32_t
let c_unit_observation = field config "unit_observation" int32_t
let c_alpha = field config "alpha" double
let c_gamma = field config "gamma" double
let c_defenders = field config "defenders" int32_t
let c_reward_scheme = field config "reward_scheme" int32_t
let c_activation_delay = field config "activation_delay" double
let c_propagation_delay = field config "propagation_delay" double
let c_max_steps = field config "max_steps" int64_t
let c_max_progress = field config "max_progress" double
let c_max_time = field config "max_time" double
let c_activations = field config "activations" int64_t
let c_seed = field config "seed" uint64_t
let c_n_lanes = field config "n_lanes" int64_t
let c_k = field config "k" int32_t
let c_subblock_selection = field config "subblock_selection" int32_t
let c_delay_lo = field config "delay_lo" double
let c_delay_hi = field config "delay_hi" double
let c_horizon = field config "horizon" double
let () = seal config

(* ---- cpr_episode_record *)
type record

let record : record structure typ = structure "cpr_episode_record"
let r_reward_attacker = field record "reward_attacker" double
let r_reward_defender = field record "reward_defender" double
let r_progress = field record "progress" double
let r_chain_time = field record "chain_time" double
let r_sim_time = field record "sim_time" double
let r_n_steps = field record "n_steps" int64_t
let r_n_activations = field record "n_activations" int64_t
let r_head_height = field record "head_height" int32_t
let r_head_miner = field record "head_miner" int32_t
let r_status = field record "status" uint32_t
let r_head_work = field record "head_work" int32_t
let () = seal record

(* ---- cpr_summary *)
let hist_bins = 64

type summary

let summary : summary structure typ = structure "cpr_summary"
let s_episodes = field summary "episodes" int64_t
let s_steps = field summary "steps" int64_t
let s_activations = field summary "activations" int64_t
let s_reward_attacker_fx = field summary "reward_attacker_fx" int64_t
let s_reward_defender_fx = field summary "reward_defender_fx" int64_t
let s_progress_fx = field summary "progress_fx" int64_t
let s_rel_revenue_fx = field summary "rel_revenue_fx" uint64_t
let s_rel_revenue_sq_fx = field summary "rel_revenue_sq_fx" uint64_t
let s_orphans = field summary "orphans" int64_t
let s_status_tie = field summary "status_tie" int64_t
let s_status_overlap = field summary "status_overlap" int64_t
let s_status_other = field summary "status_other" int64_t
let s_hist = field summary "hist" (array hist_bins int64_t)
let s_invalid = field summary "invalid" int64_t
let () = seal summary

(* ---- cpr_step_info: structure of arrays, one entry per lane *)
type step_info

let step_info : step_info structure typ = structure "cpr_step_info"
let i_episode_reward_attacker = field step_info "episode_reward_attacker" (ptr double)
let i_episode_reward_defender = field step_info "episode_reward_defender" (ptr double)
let i_episode_progress = field step_info "episode_progress" (ptr double)
let i_episode_chain_time = field step_info "episode_chain_time" (ptr double)
let i_episode_sim_time = field step_info "episode_sim_time" (ptr double)
let i_episode_n_steps = field step_info "episode_n_steps" (ptr int64_t)
let i_episode_n_activations = field step_info "episode_n_activations" (ptr int64_t)
let i_head_height = field step_info "head_height" (ptr int32_t)
let i_head_miner = field step_info "head_miner" (ptr int32_t)
let i_status = field step_info "status" (ptr uint32_t)
let () = seal step_info

(* ---- cpr_trace: CSR arrays over episodes, host memory *)
type trace

let trace : trace structure typ = structure "cpr_trace"
let t_n_episodes = field trace "n_episodes" int64_t
let t_act_offset = field trace "act_offset" (ptr int64_t)
let t_act_miner = field trace "act_miner" (ptr int32_t)
let t_act_delay = field trace "act_delay" (ptr double)
let t_pow_offset = field trace "pow_offset" (ptr int64_t)
let t_pow_hash = field trace "pow_hash" (ptr int32_t)
let t_link_offset = field trace "link_offset" (ptr int64_t)
let t_link_key = field trace "link_key" (ptr uint64_t)
let t_link_delay = field trace "link_delay" (ptr double)
let () = seal trace

(* ---- functions (include/cpr_hip.h, same order) *)
let version = foreign "cpr_version" (void @-> returning string)
let abi_version_of_library = foreign "cpr_abi_version" (void @-> returning int)
let last_error = foreign "cpr_last_error" (void @-> returning string)
let ctx_create = foreign "cpr_ctx_create" (int @-> ptr (ptr ctx) @-> returning int)
let ctx_destroy = foreign "cpr_ctx_destroy" (ptr ctx @-> returning int)
let device_count = foreign "cpr_device_count" (ptr int @-> returning int)

let batch_create =
  foreign "cpr_batch_create" (ptr ctx @-> ptr config @-> ptr (ptr batch) @-> returning int)
;;

let batch_destroy = foreign "cpr_batch_destroy" (ptr batch @-> returning int)

let run_episodes =
  foreign
    "cpr_run_episodes"
    (ptr batch @-> int64_t @-> uint64_t @-> ptr summary @-> ptr record @-> int
    @-> returning int)
;;

let run_episodes_async =
  foreign
    "cpr_run_episodes_async"
    (ptr batch @-> int64_t @-> uint64_t @-> ptr summary @-> ptr record @-> returning int)
;;

let synchronize = foreign "cpr_synchronize" (ptr ctx @-> returning int)

let replay =
  foreign
    "cpr_replay"
    (ptr batch @-> ptr trace @-> ptr summary @-> ptr record @-> int @-> returning int)
;;

let node_outputs =
  foreign
    "cpr_node_outputs"
    (ptr batch @-> int64_t @-> uint64_t @-> ptr trace @-> int32_t @-> ptr record
    @-> ptr int64_t @-> ptr double @-> returning int)
;;

let last_launch =
  foreign "cpr_last_launch" (ptr batch @-> ptr double @-> ptr int64_t @-> returning int)
;;

let launch_shape =
  foreign "cpr_launch_shape" (ptr batch @-> ptr int64_t @-> ptr int64_t @-> returning int)
;;

let rerun_hbm_retries =
  foreign "cpr_rerun_hbm_retries" (ptr ctx @-> ptr int64_t @-> returning int)
let rerun_stats =
  foreign "cpr_rerun_stats"
    (ptr ctx @-> ptr int64_t @-> ptr int64_t @-> ptr double @-> returning int)
;;

let lockstep_coverage =
  foreign "cpr_lockstep_coverage"
    (ptr batch @-> ptr int64_t @-> ptr int64_t @-> returning int)
;;

let reset =
  foreign
    "cpr_reset"
    (ptr batch @-> ptr uint8_t @-> ptr uint64_t @-> ptr double @-> returning int)
;;

let step =
  foreign
    "cpr_step"
    (ptr batch @-> ptr int32_t @-> ptr double @-> ptr double @-> ptr uint8_t
    @-> ptr step_info @-> returning int)
;;

let observe_fields = foreign "cpr_observe_fields" (ptr batch @-> ptr int32_t @-> returning int)

let rollout =
  foreign
    "cpr_rollout"
    (ptr batch @-> int64_t @-> ptr double @-> ptr double @-> ptr uint8_t @-> int
    @-> ptr summary @-> returning int)
;;

let policy_actions =
  foreign
    "cpr_policy_actions"
    (ptr batch @-> int32_t @-> ptr double @-> int64_t @-> ptr int32_t @-> returning int)
;;

let observation_spec =
  foreign
    "cpr_observation_spec"
    (ptr batch @-> ptr int32_t @-> ptr int32_t @-> ptr double @-> ptr double
    @-> returning int)
;;

let policy_count = foreign "cpr_policy_count" (int32_t @-> returning int)

let policy_name =
  foreign "cpr_policy_name" (int32_t @-> int32_t @-> ptr int32_t @-> returning string)
;;

let stream_fill =
  foreign
    "cpr_stream_fill"
    (ptr ctx @-> uint64_t @-> uint64_t @-> uint32_t @-> uint32_t @-> int64_t @-> ptr uint32_t
    @-> ptr double @-> returning int)
;;

(* errors: every entry point returns a status; non-zero becomes the exception the
   reference raises at the same point (engine.ml:37-51 Failure, network.ml:63-72
   Invalid_argument) *)
let check rc =
  if rc = e_invalid_arg
  then invalid_arg (last_error ())
  else if rc <> ok
  then failwith (Printf.sprintf "libcpr_hip (%d): %s" rc (last_error ()))
;;

let () =
  if abi_version_of_library () <> abi_version
  then
    failwith
      (Printf.sprintf
         "libcpr_hip ABI %d, bindings expect %d"
         (abi_version_of_library ())
         abi_version)
;;
