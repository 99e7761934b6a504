same as f_reconv; k_bobyqa_fit<K> templated on the dimension
