(* Hip_engine.of_module: a drop-in for Engine.of_module (simulator/gym/engine.ml:97-273)
   whose episodes run on libcpr_hip device lanes instead of the OCaml Simulator.

   Same signature and result: an AttackSpace and Engine.Parameters.t give a
   `instance ref Intf.env` (simulator/gym/intf.ml:3-13) with create / reset / step /
   to_string / policies / low / high. The attack space's own modules keep doing what only
   they know: observation decoding and printing (M.Observation), action names (M.Action),
   the policy closures (M.policies) and the protocol's Info (M.Protocol.info), from which
   the device configuration is read (family, k, incentive scheme, sub-block selection).
   The device lane reproduces engine.ml's step semantics (DESIGN.md §1-4): the info list
   has engine.ml:224-241's keys in its order, then protocol_ and head_ keys.

   To use it, cpr_gym_engine.ml's `create` (cpr_gym_engine.ml:42-89) calls
   Hip_engine.of_module where it called Engine.of_module. Built by the dune stanza next to
   this file. Not compiled here (no OCaml toolchain in this build image). *)

open Cpr_lib
open Ctypes
module H = Cpr_hip

type device_spec =
  { protocol : int32
  ; k : int32
  ; scheme : int32
  ; selection : int32
  ; unit_obs : bool
  ; obs_len : int
  ; n_act : int
  }

let lookup key (info : Info.t) =
  List.find_map (fun (k, v) -> if k = key then Some v else None) info
;;

let lookup_string key info =
  match lookup key info with
  | Some (Info.String s) -> Some s
  | _ -> None
;;

(* include/cpr_hip.h cpr_reward_scheme / cpr_subblock_selection *)
let scheme_id = function
  | "constant" -> 0l
  | "discount" -> 1l
  | "block" -> 2l
  | "punish" -> 3l
  | "hybrid" -> 4l
  | s -> invalid_arg ("Hip_engine: incentive scheme " ^ s)
;;

let selection_id = function
  | "altruistic" -> 0l
  | "heuristic" -> 1l
  | "optimal" -> 2l
  | s -> invalid_arg ("Hip_engine: sub-block selection " ^ s)
;;

(* the device protocol behind an attack space, from its Protocol.info
   (nakamoto.ml:6-9, ethereum.ml:57-64, bk.ml:21-24, tailstorm.ml:45-52) *)
let spec_of (type a) (module P : Intf.Protocol with type data = a) ~key ~obs_len ~n_act =
  let info = P.info in
  let int_ key = match lookup key info with Some (Info.Int i) -> Int32.of_int i | _ -> 8l in
  let scheme () =
    scheme_id (Option.value ~default:"constant" (lookup_string "incentive_scheme" info))
  in
  let unit_obs = String.ends_with ~suffix:"unitobs" key in
  let base = { protocol = H.proto_nakamoto; k = 8l; scheme = 0l; selection = 1l; unit_obs; obs_len; n_act } in
  match lookup_string "family" info, lookup_string "preference" info with
  | Some "nakamoto", _ -> base
  | Some "bk", _ -> { base with protocol = H.proto_bk; k = int_ "k"; scheme = scheme () }
  | Some "tailstorm", _ ->
    { base with
      protocol = H.proto_tailstorm
    ; k = int_ "k"
    ; scheme = scheme ()
    ; selection =
        selection_id
          (Option.value ~default:"heuristic" (lookup_string "subblock_selection" info))
    }
  | None, Some _ -> { base with protocol = H.proto_ethereum; scheme = scheme () }
  | _ -> invalid_arg "Hip_engine: protocol not on the device (spar/stree/sdag/tailstormjune)"
;;

(* one lane of a device batch = one gym env *)
type instance =
  { ctx : H.ctx structure ptr
  ; batch : H.batch structure ptr
  ; mutable episode : int64
  ; obs : (float, Bigarray.float64_elt) Bigarray.Array1.t
  ; mutable last : float * float * float * float * float
  }

let seed_of_env () =
  match Sys.getenv_opt "CPR_SEED" with
  | Some s -> Unsigned.UInt64.of_string s
  | None -> Unsigned.UInt64.of_int64 (Random.int64 Int64.max_int)
;;

let of_module ?(device = 0) ?seed (Intf.AttackSpace (module M)) (p : Engine.Parameters.t)
    : instance ref Intf.env
  =
  let spec =
    spec_of (module M.Protocol) ~key:M.key ~obs_len:M.Observation.length ~n_act:M.Action.n
  in
  let seed = match seed with Some s -> s | None -> seed_of_env () in
  let cfg = make H.config in
  setf cfg H.c_protocol spec.protocol;
  setf cfg H.c_network H.net_selfish_mining;
  setf cfg H.c_mode H.mode_gym;
  setf cfg H.c_policy 0l;
  setf cfg H.c_policy_table (from_voidp uint8_t null);
  setf cfg H.c_policy_table_dim 0l;
  setf cfg H.c_unit_observation (if spec.unit_obs then 1l else 0l);
  setf cfg H.c_alpha p.alpha;
  setf cfg H.c_gamma p.gamma;
  setf cfg H.c_defenders (Int32.of_int p.defenders);
  setf cfg H.c_reward_scheme spec.scheme;
  setf cfg H.c_activation_delay p.activation_delay;
  setf cfg H.c_propagation_delay 1e-9 (* engine.ml:100-107 *);
  setf cfg H.c_max_steps (Int64.of_int p.max_steps);
  setf cfg H.c_max_progress (if p.max_progress < infinity then p.max_progress else 0.);
  setf cfg H.c_max_time (if p.max_time < infinity then p.max_time else 0.);
  setf cfg H.c_activations 0L;
  setf cfg H.c_seed seed;
  setf cfg H.c_n_lanes 1L;
  setf cfg H.c_k spec.k;
  setf cfg H.c_subblock_selection spec.selection;
  setf cfg H.c_delay_lo Float.nan;
  setf cfg H.c_delay_hi Float.nan;
  setf cfg H.c_horizon 100.;
  let new_instance () =
    let c = allocate (ptr H.ctx) (from_voidp H.ctx null) in
    H.check (H.ctx_create device c);
    let b = allocate (ptr H.batch) (from_voidp H.batch null) in
    H.check (H.batch_create !@c (addr cfg) b);
    Gc.finalise
      (fun _ ->
        ignore (H.batch_destroy !@b);
        ignore (H.ctx_destroy !@c))
      b;
    { ctx = !@c
    ; batch = !@b
    ; episode = 0L
    ; obs = Bigarray.(Array1.create float64 c_layout spec.obs_len)
    ; last = 0., 0., 0., 0., 0.
    }
  in
  let floatarray_of_obs t = Float.Array.init spec.obs_len (fun i -> t.obs.{i}) in
  (* engine.ml:164-170: a fresh episode; here the next episode id of the lane's stream *)
  let reset ref_t =
    let t = !ref_t in
    let eps = allocate uint64_t (Unsigned.UInt64.of_int64 t.episode) in
    t.episode <- Int64.succ t.episode;
    t.last <- 0., 0., 0., 0., 0.;
    H.check (H.reset t.batch (from_voidp uint8_t null) eps (bigarray_start array1 t.obs));
    floatarray_of_obs t
  in
  let create () = ref (new_instance ()) in
  let step ref_t ~action =
    let t = !ref_t in
    if action < 0 || action >= spec.n_act then invalid_arg "index out of bounds";
    let a = allocate int32_t (Int32.of_int action) in
    let reward = allocate double 0. and done_ = allocate uint8_t Unsigned.UInt8.zero in
    let info = make H.step_info in
    let d f = let x = allocate double 0. in setf info f x; x in
    let i64 f = let x = allocate int64_t 0L in setf info f x; x in
    let i32 f = let x = allocate int32_t 0l in setf info f x; x in
    let era = d H.i_episode_reward_attacker and erd = d H.i_episode_reward_defender
    and prog = d H.i_episode_progress and ct = d H.i_episode_chain_time
    and st = d H.i_episode_sim_time and steps = i64 H.i_episode_n_steps
    and acts = i64 H.i_episode_n_activations and hh = i32 H.i_head_height
    and hm = i32 H.i_head_miner in
    let status = allocate uint32_t Unsigned.UInt32.zero in
    setf info H.i_status status;
    H.check
      (H.step t.batch a (bigarray_start array1 t.obs) reward done_ (addr info));
    let status = Unsigned.UInt32.to_int32 !@status in
    if Int32.logand status H.st_reference_raises <> 0l
    then failwith "the reference simulator raises an exception at this step";
    if Int32.logand status H.st_capacity <> 0l
    then failwith "device lane capacity exceeded";
    let ra, rd, pr, ctm, stm = !@era, !@erd, !@prog, !@ct, !@st in
    let la, ld, lp, lc, ls = t.last in
    t.last <- ra, rd, pr, ctm, stm;
    let head =
      let open Info in
      let miner = Int32.to_int !@hm in
      match spec.protocol with
      | x when x = H.proto_nakamoto ->
        (* nakamoto.ml:22-27 *)
        [ int "height" (Int32.to_int !@hh)
        ; string "miner" (if miner < 0 then "n/a" else string_of_int miner)
        ]
      | x when x = H.proto_ethereum ->
        (* ethereum.ml:92-95 *)
        [ int "height" (Int32.to_int !@hh); int "work" (int_of_float pr) ]
      | x when x = H.proto_bk -> [ string "kind" "block"; int "height" (Int32.to_int !@hh) ]
      | _ -> [ string "kind" "summary"; int "height" (Int32.to_int !@hh) ]
    in
    let info =
      let open Info in
      [ float "step_reward_attacker" (ra -. la)
      ; float "step_reward_defender" (rd -. ld)
      ; float "step_progress" (pr -. lp)
      ; float "step_chain_time" (ctm -. lc)
      ; float "step_sim_time" (stm -. ls)
      ; float "episode_reward_attacker" ra
      ; float "episode_reward_defender" rd
      ; float "episode_progress" pr
      ; float "episode_chain_time" ctm
      ; float "episode_sim_time" stm
      ; int "episode_n_steps" (Int64.to_int !@steps)
      ; int "episode_n_activations" (Int64.to_int !@acts)
      ]
      @ Info.prefix_key "protocol_" M.Protocol.info
      @ Info.prefix_key "head_" head
      @
      if Int32.logand status H.st_lockstep_inexact <> 0l
      then [ int "device_status" (Int32.to_int status) ]
      else []
    in
    floatarray_of_obs t, !@reward, Unsigned.UInt8.to_int !@done_ <> 0, info
  in
  let actions_hum =
    List.init M.Action.n (fun i -> Printf.sprintf "(%d) %s" i M.Action.(of_int i |> to_string))
    |> String.concat " | "
  in
  (* engine.ml:250-257 *)
  let to_string ref_t =
    let t = !ref_t in
    Printf.sprintf
      "%s; %s; α=%.2f attacker\n%s\nActions: %s"
      M.Protocol.description
      M.info
      p.alpha
      (floatarray_of_obs t |> M.Observation.of_floatarray |> M.Observation.to_string)
      actions_hum
  in
  (* engine.ml:258-261: the attack space's own policy closures *)
  let policies =
    Collection.map_to_list
      (fun e -> e.key, fun a -> M.Observation.of_floatarray a |> e.it |> M.Action.to_int)
      M.policies
  in
  { Intf.n_actions = M.Action.n
  ; observation_length = M.Observation.length
  ; create
  ; reset
  ; step
  ; low = M.Observation.low
  ; high = M.Observation.high
  ; to_string
  ; policies
  }
;;
