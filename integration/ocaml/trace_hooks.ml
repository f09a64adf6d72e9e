(* Trace recording for the reference simulator (simulator/lib/simulator.ml), so that the
   OCaml engine can export the activation / delay trace of an episode and libcpr_hip can
   replay the very same draws (cpr_replay, include/cpr_hip.h `cpr_trace`; DESIGN.md §3.1).

   UNCOMPILED HERE: this build image has no OCaml toolchain (SURVEY.md §8c). The module
   uses only the standard library (OCaml >= 4.08 for Bytes.set_int64_le); the hooks are
   inserted by simulator_trace.patch. Recording is off unless a recorder is installed
   (`start`), so simulations that do not export traces are unchanged.

   Draw coordinates (the keyed-stream coordinates of cpr_amd/csrc/cpr_stream.h):
   - act_miner[k]  miner of activation k (k = clock.c_activations before the increment),
                   StochasticClock, simulator.ml:465-472
   - act_delay[j]  exponential delay of clock j (j = clock.c_activations when drawn; the
                   first clock of init is j = 0), schedule_proof_of_work
   - pow_hash[s]   Random.bits of the PoW vertex with serial s, raw_append,
                   simulator.ml:122-136
   - link delays   one per (message, outgoing link) drawn at Network Tx,
                   simulator.ml:481-487, keyed
                     (kw lsl 32) lor (off lsl 12) lor dest   Nakamoto / Ethereum: kw =
                        c_activations when the share happened, off = the message's position
                        in that handle_action's recursive share (simulator.ml:401-419)
                     (serial lsl 32) lor dest                B_k / Tailstorm (by vertex)
                   constant-delay links draw nothing and are not recorded.
   A draw at a coordinate drawn before (the gym's reset runs Simulator.init twice,
   engine.ml:164-170) overwrites it, as the oracle's recorder does (oracle/src/des.cpp). *)

type link_keys =
  | By_share  (** Nakamoto, Ethereum *)
  | By_serial  (** B_k, Tailstorm *)

(* growable arrays with overwrite-at-index semantics *)
module Vec = struct
  type 'a t =
    { mutable a : 'a array
    ; mutable n : int
    ; fill : 'a
    }

  let create fill = { a = Array.make 64 fill; n = 0; fill }
  let clear v = v.n <- 0

  let put v i x =
    if i >= Array.length v.a
    then (
      let b = Array.make (max (i + 1) (2 * Array.length v.a)) v.fill in
      Array.blit v.a 0 b 0 v.n;
      v.a <- b);
    if i >= v.n
    then (
      Array.fill v.a v.n (i + 1 - v.n) v.fill;
      v.n <- i + 1);
    v.a.(i) <- x
  ;;

  let to_list v = Array.to_list (Array.sub v.a 0 v.n)
end

type episode =
  { miner : int Vec.t
  ; delay : float Vec.t
  ; pow : int Vec.t
  ; links : (int, float) Hashtbl.t  (** key -> delay *)
  ; shares : (int * int, int * int) Hashtbl.t  (** (node, vertex id) -> (kw, off) *)
  ; mutable share_off : int
  }

type t =
  { keys : link_keys
  ; ep : episode
  ; (* finished episodes, CSR (arrays of cpr_trace in cpr_amd._lib.Trace.ARRAYS order) *)
    mutable act_offset : int list
  ; mutable act_miner : int list list
  ; mutable act_delay : float list list
  ; mutable pow_offset : int list
  ; mutable pow_hash : int list list
  ; mutable link_offset : int list
  ; mutable link_key : int list list
  ; mutable link_delay : float list list
  }

let create keys =
  { keys
  ; ep =
      { miner = Vec.create 0
      ; delay = Vec.create 0.
      ; pow = Vec.create 0
      ; links = Hashtbl.create 256
      ; shares = Hashtbl.create 256
      ; share_off = 0
      }
  ; act_offset = [ 0 ]
  ; act_miner = []
  ; act_delay = []
  ; pow_offset = [ 0 ]
  ; pow_hash = []
  ; link_offset = [ 0 ]
  ; link_key = []
  ; link_delay = []
  }
;;

(* the recorder the hooks write to; None = recording off (the default) *)
let current : t option ref = ref None
let start t = current := Some t
let stop () = current := None
let with_rec f = Option.iter f !current

(* ---- hooks (called from simulator.ml, see simulator_trace.patch) *)

(* StochasticClock: the miner of activation k *)
let record_miner ~k node = with_rec (fun t -> Vec.put t.ep.miner k node)

(* schedule_proof_of_work: the delay of clock j *)
let record_delay ~j d = with_rec (fun t -> Vec.put t.ep.delay j d)

(* raw_append: the 30-bit PoW hash of the vertex with this serial *)
let record_pow ~serial bits = with_rec (fun t -> Vec.put t.ep.pow serial bits)

(* handle_action: a new recursive share starts (message positions restart at 0) *)
let begin_share () = with_rec (fun t -> t.ep.share_off <- 0)

(* handle_action's share: vertex [id] is released by [node] at activation count [kw] *)
let note_share ~node ~id ~kw =
  with_rec (fun t ->
    Hashtbl.replace t.ep.shares (node, id) (kw, t.ep.share_off);
    t.ep.share_off <- t.ep.share_off + 1)
;;

let link_key_share ~kw ~off ~dest = (kw lsl 32) lor ((off land 0xFFFFF) lsl 12) lor (dest land 0xFFF)
let link_key_serial ~serial ~dest = (serial lsl 32) lor (dest land 0xFFF)

(* Network Tx: the delay drawn for the link src -> dest of vertex [id] (its DAG serial).
   [constant] links draw nothing and are skipped. *)
let record_tx ~src ~id ~dest ~constant d =
  with_rec (fun t ->
    if not constant
    then (
      let key =
        match t.keys with
        | By_serial -> link_key_serial ~serial:id ~dest
        | By_share ->
          (match Hashtbl.find_opt t.ep.shares (src, id) with
           | Some (kw, off) -> link_key_share ~kw ~off ~dest
           | None -> invalid_arg "Trace_hooks.record_tx: message was never shared")
      in
      Hashtbl.replace t.ep.links key d))
;;

(* ---- episodes *)

(* close the running episode: append its draws (links sorted by key, as the device's
   binary search expects) and start an empty one *)
let end_episode t =
  let e = t.ep in
  let last l = List.hd l in
  t.act_miner <- Vec.to_list e.miner :: t.act_miner;
  t.act_delay <- Vec.to_list e.delay :: t.act_delay;
  t.act_offset <- (last t.act_offset + max e.miner.n e.delay.n) :: t.act_offset;
  t.pow_hash <- Vec.to_list e.pow :: t.pow_hash;
  t.pow_offset <- (last t.pow_offset + e.pow.n) :: t.pow_offset;
  let links = Hashtbl.fold (fun k d acc -> (k, d) :: acc) e.links [] in
  let links = List.sort (fun (a, _) (b, _) -> compare a b) links in
  t.link_key <- List.map fst links :: t.link_key;
  t.link_delay <- List.map snd links :: t.link_delay;
  t.link_offset <- (last t.link_offset + List.length links) :: t.link_offset;
  Vec.clear e.miner;
  Vec.clear e.delay;
  Vec.clear e.pow;
  Hashtbl.reset e.links;
  Hashtbl.reset e.shares;
  e.share_off <- 0
;;

(* ---- binary writer (read by cpr_amd._lib.Trace.load)

   "CPRTRACE" | u32 version = 1 | u32 n_episodes | then the eight arrays of
   Trace.ARRAYS in order, each: u64 count | count little-endian elements
     act_offset i64 | act_miner i32 | act_delay f64 | pow_offset i64 | pow_hash i32 |
     link_offset i64 | link_key u64 | link_delay f64
   act_miner and act_delay have one entry per activation index: an index the episode did
   not draw (a miner past the last activation) is written as 0. *)

let write path t =
  let buf = Buffer.create (1 lsl 16) in
  let b8 = Bytes.create 8 in
  let u32 x =
    Bytes.set_int32_le b8 0 (Int32.of_int x);
    Buffer.add_subbytes buf b8 0 4
  in
  let i64 x =
    Bytes.set_int64_le b8 0 (Int64.of_int x);
    Buffer.add_subbytes buf b8 0 8
  in
  let f64 x =
    Bytes.set_int64_le b8 0 (Int64.bits_of_float x);
    Buffer.add_subbytes buf b8 0 8
  in
  let arr put xs =
    i64 (List.length xs);
    List.iter put xs
  in
  let csr xss = List.concat (List.rev xss) in
  (* per episode, miners and delays padded to the same length *)
  let pad fill n xs = xs @ List.init (max 0 (n - List.length xs)) (fun _ -> fill) in
  let lens =
    List.rev (List.map2 (fun m d -> max (List.length m) (List.length d)) t.act_miner t.act_delay)
  in
  let miners = List.map2 (pad 0) lens (List.rev t.act_miner) in
  let delays = List.map2 (pad 0.) lens (List.rev t.act_delay) in
  Buffer.add_string buf "CPRTRACE";
  u32 1;
  u32 (List.length t.act_offset - 1);
  arr i64 (List.rev t.act_offset);
  arr u32 (List.concat miners);
  arr f64 (List.concat delays);
  arr i64 (List.rev t.pow_offset);
  arr u32 (csr t.pow_hash);
  arr i64 (List.rev t.link_offset);
  arr i64 (csr t.link_key);
  arr f64 (csr t.link_delay);
  let oc = open_out_bin path in
  Buffer.output_buffer oc buf;
  close_out oc
;;
