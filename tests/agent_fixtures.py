"""Shared scenario for the agent-loop parity test and its golden-vector generator
(tools/gen_golden_agent.py): an offline character-level tokenizer with a Qwen-style chat
template, a scripted inference client, and a small sqlite database. Pure data and plumbing:
nothing here is the code under test."""

import os
import sqlite3

CHAT_TEMPLATE = ("{% for m in messages %}<|im_start|>{{ m['role'] }}\n{{ m['content'] }}<|im_end|>\n{% endfor %}"
                 "{% if add_generation_prompt %}<|im_start|>assistant\n{% endif %}")
SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]


def make_tokenizer():
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast

    chars = [chr(c) for c in range(32, 127)] + ["\n", "\t"]
    vocab = {s: i for i, s in enumerate(SPECIALS + chars + ["<unk>"])}
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Split(Regex(r"[\s\S]"), behavior="isolated")
    tk.decoder = decoders.Fuse()
    class ListChatTokenizer(PreTrainedTokenizerFast):
        # transformers 4.x behaviour (what the reference generator is written against):
        # apply_chat_template(tokenize=True) returns the id list, not a BatchEncoding
        def apply_chat_template(self, conversation, **kw):
            if kw.get("tokenize", True):
                kw.setdefault("return_dict", False)
            return super().apply_chat_template(conversation, **kw)

    t = ListChatTokenizer(tokenizer_object=tk, eos_token="<|im_end|>", pad_token="<|endoftext|>",
                          unk_token="<unk>", additional_special_tokens=SPECIALS)
    t.chat_template = CHAT_TEMPLATE
    return t


DB_ROWS = [(1, "alice", 34), (2, "bob", 27), (3, "carol", 41)]


def make_sql_root(root):
    """{root}/spider/database/people/people.sqlite with one table."""
    d = os.path.join(root, "spider", "database", "people")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "people.sqlite")
    if os.path.exists(path):
        os.remove(path)
    con = sqlite3.connect(path)
    con.execute("CREATE TABLE person (id INTEGER, name TEXT, age INTEGER)")
    con.executemany("INSERT INTO person VALUES (?, ?, ?)", DB_ROWS)
    con.commit()
    con.close()
    return root


# session -> scripted turns: (text, stop_reason, ends_with_eos)
SCRIPTS = {
    "sql_ok_0": [("<think>look up bob</think><sql>SELECT age FROM person WHERE name = 'bob'</sql>", "stop", False),
                 ("<think>it is 27</think><solution>SELECT age FROM person WHERE id = 2</solution>", "stop", False)],
    "sql_bad_0": [("<think>hmm</think> no tool call here", "stop", True),
                  ("<think>try</think><sql>SELECT nonexistent FROM person</sql>", "stop", False),
                  ("<think>guess</think><solution>SELECT 99</solution>", "stop", False)],
    "sql_turns_0": [("<think>a</think><sql>SELECT COUNT(*) FROM person</sql>", "stop", False),
                    ("<think>b</think><sql>SELECT MAX(age) FROM person</sql>", "stop", False),
                    ("<think>c</think><sql>SELECT MIN(age) FROM person</sql>", "stop", False)],
    "sql_fmt_0": [("<solution>SELECT age FROM person WHERE id = 2</solution>", "stop", False)],
    "sql_len_0": [("<think>" + "x" * 450 + "</think><sql>SELECT 1</sql>", "length", False)],
    "gsm_ok_0": [("6 * 7 = 42\n#### 42", "stop", True)],
    "gsm_bad_0": [("the answer is 41 #### 41", "stop", True)],
    "gsm_trunc_0": [("so far 4", "length", False)],
}


# the reply once a session's script is exhausted (the re-tokenizing mode checks the input length
# before adding a turn, so a length-cut trajectory asks for one more turn)
EXTRA_TURN = ("<think>more</think><solution>SELECT 1</solution>", "stop", False)


class ScriptedClient:
    """InferenceEngineClient stand-in: per session id, returns the next scripted turn (token ids
    through the shared tokenizer; eos appended when the script says the engine stopped on it).
    Text-in requests ("prompts": conversations, the batched generator) are answered per
    conversation with the first turn of the script named by the last message's "<name>:" prefix.
    logprobs=False leaves response_logprobs out, as an engine asked for no logprobs does."""

    def __init__(self, tokenizer, logprobs=True):
        self.tok = tokenizer
        self.turn = {}
        self.prompts = []
        self.logprobs = logprobs

    def _reply(self, text, reason, with_eos):
        ids = self.tok.encode(text, add_special_tokens=False)
        if with_eos:
            ids = ids + [self.tok.eos_token_id]
            text = text + self.tok.eos_token
        return text, ids, reason, [-0.01 * (i + 1) for i in range(len(ids))]

    async def generate(self, inp):
        if inp.get("prompts") is not None:
            outs = []
            for conv in inp["prompts"]:
                name = conv[-1]["content"].split(":")[0].split()[-1]
                self.prompts.append((name, [m["content"] for m in conv]))
                outs.append(self._reply(*SCRIPTS[f"{name}_0"][0]))
            res = {"responses": [o[0] for o in outs], "response_ids": [o[1] for o in outs],
                   "stop_reasons": [o[2] for o in outs]}
            if self.logprobs:
                res["response_logprobs"] = [o[3] for o in outs]
            return res
        sid = inp["session_ids"][0]
        k = self.turn.get(sid, 0)
        self.turn[sid] = k + 1
        script = SCRIPTS[sid]
        text, reason, with_eos = script[k] if k < len(script) else EXTRA_TURN
        self.prompts.append((sid, list(inp["prompt_token_ids"][0])))
        out_text, ids, reason, lps = self._reply(text, reason, with_eos)
        res = {"responses": [out_text], "response_ids": [ids], "stop_reasons": [reason]}
        if self.logprobs:
            res["response_logprobs"] = [lps]
        return res


# generator-mode cases beyond the two chat modes (tools/gen_golden_agent.py MODE_CASES):
#   name -> GeneratorConfig overrides, whether the engine returns logprobs, scenario subset
MODE_CASES = {
    "retokenize_qwen3_without_thinking": (dict(use_conversation_multi_turn=True,
                                               chat_template={"source": "name",
                                                              "name_or_path": "qwen3_without_thinking"}),
                                          False, "all"),
    "retokenize_qwen3_with_thinking": (dict(use_conversation_multi_turn=True,
                                            chat_template={"source": "name", "name_or_path": "qwen3_with_thinking"}),
                                       False, "all"),
    "custom_template_single_turn_chat": (dict(use_conversation_multi_turn=False,
                                              chat_template={"source": "name",
                                                             "name_or_path": "qwen3_without_thinking"}),
                                         False, "all"),
    "step_wise": (dict(use_conversation_multi_turn=True, step_wise_trajectories=True), True, "all"),
    "step_wise_flags": (dict(use_conversation_multi_turn=True, step_wise_trajectories=True,
                             zero_reward_on_non_stop=True, apply_overlong_filtering=True), True, "all"),
    "batched": (dict(batched=True, use_conversation_multi_turn=False), True, "single_turn"),
    "batched_overlong": (dict(batched=True, use_conversation_multi_turn=False, apply_overlong_filtering=True),
                         True, "single_turn"),
}


def scenario_subset(multi_turn, subset):
    prompts, classes, extras, tids = scenario(multi_turn)
    if subset == "single_turn":  # the GSM8K trajectories (one turn each)
        keep = [i for i, c in enumerate(classes) if c == "gsm8k"]
        return ([prompts[i] for i in keep], [classes[i] for i in keep], [extras[i] for i in keep],
                [tids[i] for i in keep])
    return prompts, classes, extras, tids


def scenario(multi_turn):
    """GeneratorInput pieces (plain data) for one batch of 8 trajectories."""
    sys_msg = {"role": "system", "content": "Answer with SQL."}
    prompts, classes, extras, tids = [], [], [], []
    for name in ("sql_ok", "sql_bad", "sql_turns", "sql_fmt", "sql_len"):
        prompts.append([sys_msg, {"role": "user", "content": f"Task {name}: how old is bob?"}])
        classes.append("text2sql")
        extras.append({"db_id": "people", "data": "spider",
                       "reward_spec": {"ground_truth": "SELECT age FROM person WHERE name = 'bob'"}})
        tids.append((name, 0))
    for name, gt in (("gsm_ok", "42"), ("gsm_bad", "42"), ("gsm_trunc", "4")):
        prompts.append([{"role": "user", "content": f"{name}: what is 6*7?"}])
        classes.append("gsm8k")
        extras.append({"reward_spec": {"method": "rule", "ground_truth": gt}})
        tids.append((name, 0))
    return prompts, classes, extras, tids
