same as f_reconv; BOBYQA evaluations through css_pass<P,Q,I>
